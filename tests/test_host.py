"""Host-side logic on CPU: EpisodeBatch / ReplayBuffer semantics against the reference's golden vectors,
env-spec construction from match build plans, PFSP/payoff helpers."""
import numpy as np
import pytest
import torch

from helpers import qmix_args, scheme_for


def _mk_batch(B, T, N, d_obs, A, S, lengths, seed):
    """Same construction as tests/golden/make_golden.py::make_batch, through maleague.EpisodeBatch."""
    from maleague.components.episode_batch import EpisodeBatch
    info = {"state_shape": S, "obs_shape": d_obs, "n_actions": A, "n_agents": N}
    scheme, groups, preprocess = scheme_for(info, torch)
    batch = EpisodeBatch(scheme, groups, B, T, preprocess=preprocess, device="cpu")
    rng = np.random.RandomState(seed)
    for b, L in enumerate(lengths):
        for t in range(min(L + 1, T)):
            avail = (rng.rand(N, A) < 0.6).astype(np.int32)
            for n in range(N):
                if avail[n].sum() == 0:
                    avail[n, rng.randint(A)] = 1
            acts = np.array([[rng.choice(np.nonzero(avail[n])[0])] for n in range(N)], dtype=np.int64)
            pre = {"state": [rng.randn(S).astype(np.float32).tolist()], "avail_actions": [avail.tolist()],
                   "obs": [rng.randn(N, d_obs).astype(np.float32).tolist()]}
            batch.update(pre, bs=[b], ts=t, mark_filled=True)
            batch.update({"actions": torch.tensor(acts).unsqueeze(0)}, bs=[b], ts=t, mark_filled=False)
            if t < L:
                batch.update({"reward": [(float(rng.randn()),)], "terminated": [(t == L - 1,)]}, bs=[b], ts=t,
                             mark_filled=False)
    return batch, scheme, groups, preprocess


def test_episode_batch_matches_golden_learner_batch(golden):
    d = golden("qlearner_qmix_dq.npz")
    batch, *_ = _mk_batch(4, 7, 5, 80, 15, 60, [6, 3, 4, 2], seed=8)
    for k, v in batch.data.transition_data.items():
        np.testing.assert_array_equal(v.numpy(), d[f"b.{k}"], err_msg=k)
    assert int(batch.max_t_filled()) == 7
    sub = batch[:, :3]
    assert sub.max_seq_length == 3 and sub["obs"].shape[1] == 3
    assert batch[[0, 2]]["obs"].shape[0] == 2
    view = batch[("obs", "reward")]
    assert set(view.data.transition_data) == {"obs", "reward"}
    with pytest.raises(KeyError):
        batch.update({"nope": [1]}, ts=0)


def test_replay_buffer_matches_golden(golden):
    from maleague.components.replay_buffer import ReplayBuffer
    d = golden("replay_buffer.npz")
    B, T, N, d_obs, A, S = 3, 5, 5, 8, 4, 6
    info = {"state_shape": S, "obs_shape": d_obs, "n_actions": A, "n_agents": N}
    scheme, groups, preprocess = scheme_for(info, torch)
    buf = ReplayBuffer(scheme, groups, 7, T, preprocess=preprocess, device="cpu")
    for k in range(4):
        batch, *_ = _mk_batch(B, T, N, d_obs, A, S, [4 - k % 2, 2 + k % 3, 1 + k], seed=10 + k)
        np.testing.assert_array_equal(batch["obs"].numpy(), d[f"ins{k}.obs"])
        buf.insert_episode_batch(batch)
        assert buf.buffer_index == int(d[f"after{k}.buffer_index"])
        assert buf.episodes_in_buffer == int(d[f"after{k}.episodes_in_buffer"])
        np.testing.assert_array_equal(buf["obs"].numpy(), d[f"after{k}.obs"])
        np.testing.assert_array_equal(buf["filled"].numpy(), d[f"after{k}.filled"])
        np.testing.assert_array_equal(buf["actions_onehot"].numpy(), d[f"after{k}.actions_onehot"])
    assert int(buf.max_t_filled()) == int(d["max_t_filled"])
    buf2 = ReplayBuffer(scheme, groups, 3, T, preprocess=preprocess, device="cpu")
    batch, *_ = _mk_batch(B, T, N, d_obs, A, S, [2, 3, 1], seed=20)
    buf2.insert_episode_batch(batch)
    smp = buf2.sample(3)
    np.testing.assert_array_equal(smp["obs"].numpy(), d["full_sample.obs"])
    assert int(smp.max_t_filled()) == int(d["full_sample.max_t"])
    assert buf.can_sample(7) and not buf.can_sample(8)
    s = buf.sample(4)
    assert s.batch_size == 4


@pytest.mark.parametrize("plan,U,N", [("small", 6, 3), ("medium_1h_4t", 10, 5), ("large", 50, 25)])
def test_spec_from_builtin_plans(plan, U, N):
    from maleague.envs.teams_env import TeamsEnvSpec
    s = TeamsEnvSpec.from_env_args({"match_build_plan": plan, "grid_size": 20})
    assert s.U == U and s.n_agents == N and s.n_actions == 5 + U
    assert s.env_info() == {"n_agents": N, "n_actions": 5 + U, "state_shape": 6 * U, "obs_shape": 8 * U,
                            "episode_limit": 100}
    assert s.policy_team == 1 and s.agent_unit == list(range(U // 2, U))
    c = s.to_c()
    assert c.U == U and c.n_agents == N and list(c.agent_unit[:N]) == s.agent_unit


def test_spec_reads_reference_json_format(tmp_path):
    """A config/teams/<plan>.json in the reference's enum-encoded format is read as-is."""
    import json
    from maleague.envs.plans import builtin_plan
    from maleague.envs.teams_env import TeamsEnvSpec
    plan = builtin_plan("medium_1h_2t_2a_melee")
    (tmp_path / "teams").mkdir()
    (tmp_path / "teams" / "custom.json").write_text(json.dumps(plan))
    s = TeamsEnvSpec.from_env_args({"match_build_plan": "custom"}, config_dir=str(tmp_path))
    assert s.role[:5] == [0, 0, 1, 2, 2] and s.melee == [1] * 10
    s2 = TeamsEnvSpec.from_env_args({"match_build_plan": builtin_plan("small", self_play=True)})
    assert s2.n_agents == 6 and s2.n_policy_teams == 2 and s2.policy_team == 0
    with pytest.raises(FileNotFoundError):
        TeamsEnvSpec.from_env_args({"match_build_plan": "nonexistent"})


def test_env_oracle_self_consistency():
    """The C oracle keeps every agent's availability non-empty and terminates by episode_limit."""
    import envref
    from maleague.envs.teams_env import TeamsEnvSpec
    s = TeamsEnvSpec.from_env_args({"match_build_plan": "medium_1h_2t_2a", "episode_limit": 30})
    e = envref.RefEnv(s.team, s.role, s.melee, s.scripted, episode_limit=30, seed=1, env_index=3)
    rng = np.random.RandomState(0)
    for ep in range(5):
        e.reset()
        for t in range(30):
            av = e.avail()
            assert (av.sum(1) >= 1).all()
            _, done, info = e.step([rng.choice(np.nonzero(av[n])[0]) for n in range(e.N)])
            if done:
                assert t < 29 or True
                break
        assert done


def test_stepper_two_runs_before_insert_keep_the_ring_intact(monkeypatch):
    """a second train-mode run() before insert_episode_batch must not overwrite the first run's
    episodes (which the zero-copy path writes straight into the ring's next slots): it goes to a fresh batch,
    like the reference, whose buffer is untouched until insert. The kernel launch is replaced by a fake that
    stamps each run's id into its target (CPU: no GPU calls)."""
    from types import SimpleNamespace
    from maleague.components.replay_buffer import ReplayBuffer, RingEpisodeBatch
    from maleague.components.epsilon_schedules import DecayThenFlatSchedule
    from maleague.custom_logging import MainLogger
    from maleague.steppers import ParallelStepper
    import maleague.steppers.parallel_stepper as ps

    class _Ev:
        def record(self):
            pass

        def synchronize(self):
            pass

    monkeypatch.setattr(ps.torch.cuda, "Event", lambda *a, **k: _Ev())
    B, T = 4, 11
    args = qmix_args(batch_size_run=B, device="cpu", env_args={"match_build_plan": "medium_1h_4t", "grid_size": 20,
                                                               "stochastic_spawns": True, "episode_limit": T - 1})
    stepper = ParallelStepper(args, MainLogger())
    info = stepper.get_env_info()
    scheme, groups, preprocess = scheme_for(info, torch)
    sel = SimpleNamespace(schedule=DecayThenFlatSchedule(1.0, 0.05, 50000), epsilon=1.0)
    stepper.initialize(scheme, groups, preprocess, SimpleNamespace(init_hidden=lambda batch_size: None,
                                                                   action_selector=sel))
    ring = ReplayBuffer(scheme, groups, 10, T, preprocess=preprocess, device="cpu")
    assert stepper.attach_replay(ring)
    stamp = [0]

    def fake_to_mlg(batch):
        return SimpleNamespace(target=batch, B=B, ring_slot0=0, ring_size=0, full_write=0), []

    def fake_launch(mb, eps, test_mode):
        stamp[0] += 1
        obs = mb.target.data.transition_data["obs"]
        if mb.target is ring:  # kernel writes slots [ring_slot0, +B) mod size
            for b in range(mb.B):
                obs[(mb.ring_slot0 + b) % mb.ring_size].fill_(stamp[0])
        else:
            obs.fill_(stamp[0])
        stepper._info[0:B] = 3

    monkeypatch.setattr(stepper, "_to_mlg", fake_to_mlg)
    monkeypatch.setattr(stepper, "_launch_mb", fake_launch)
    b1, _ = stepper.run(test_mode=False)
    assert isinstance(b1, RingEpisodeBatch) and ring.has_outstanding()
    b2, _ = stepper.run(test_mode=False)  # second run before any insert: fresh batch, ring untouched
    assert not isinstance(b2, RingEpisodeBatch)
    assert (b1["obs"] == 1).all() and (b2["obs"] == 2).all()
    ring.insert_episode_batch(b1)
    ring.insert_episode_batch(b2)
    assert (ring["obs"][0:B] == 1).all() and (ring["obs"][B:2 * B] == 2).all()
    assert ring.buffer_index == 2 * B and not ring.has_outstanding()
    # back to the zero-copy path once nothing is outstanding
    b3, _ = stepper.run(test_mode=False)
    assert isinstance(b3, RingEpisodeBatch) and b3.slot0 == 2 * B
    # inserting a plain batch first detaches the uncommitted ring episodes before their slots are overwritten
    b4, _ = stepper.run(test_mode=False)
    ring.insert_episode_batch(b4)
    assert not b3.attached and (b3["obs"] == 3).all()
    ring.insert_episode_batch(b3)
    # b4 took slots 8, 9, 0, 1 (wrap at 10), b3 the next four
    assert (ring["obs"][8:10] == 4).all() and (ring["obs"][0:2] == 4).all() and (ring["obs"][2:6] == 3).all()


class _BoundsStepper:
    """A stepper whose runs resolve lazily: t_env advances by `lens[i]` per run, known exactly only after a resolve
    (ParallelStepper's run-ahead); bounds = (resolved, resolved + limit per run in flight)."""

    def __init__(self, lens, limit=100, B=4):
        self.lens, self.limit, self.batch_size = list(lens), limit, B
        self._t = 0
        self._pending = []
        self.resolves = 0

    def run(self):
        self._pending.append(self.lens.pop(0))

    def t_env_bounds(self):
        return self._t, self._t + len(self._pending) * self.batch_size * self.limit

    @property
    def t_env(self):
        if self._pending:
            self.resolves += 1
        self._t += sum(self._pending) * self.batch_size
        self._pending = []
        return self._t


def test_loop_interval_checks_resolve_only_at_thresholds():
    """MultiAgentExperiment's t_max / test / save / log checks answer exactly as with the exact t_env, and
    resolve the runs in flight only when the bounds of t_env straddle a threshold."""
    from types import SimpleNamespace
    from maleague.runs.ma_experiment import MultiAgentExperiment

    def run_loop(lens, exact):
        st = _BoundsStepper(lens)
        exp = MultiAgentExperiment.__new__(MultiAgentExperiment)
        exp.args = SimpleNamespace(test_interval=2000, log_interval=3000, save_model=True, save_model_interval=5000,
                                   test_nepisode=4, batch_size_run=4, t_max=10 ** 9)
        exp.stepper, exp.last_test_T, exp.last_log_T, exp.model_save_time = st, -2001, 0, 0
        events = []
        exp._train_episode = lambda episode_num: st.run()
        exp._test = lambda n: (events.append(("test", st.t_env)), setattr(exp, "last_test_T", st.t_env))
        exp.save_models = lambda: (events.append(("save", st.t_env)), setattr(exp, "model_save_time", st.t_env))
        exp.logger = SimpleNamespace(log_stat=lambda k, v, t: events.append(("log", t)))
        if exact:  # reference semantics: the exact t_env at every check
            exp._t_env_reached = lambda thr: st.t_env >= thr
        ep = 0
        for _ in range(len(lens)):
            ep = exp._iteration(ep)
            if exact:
                _ = st.t_env
        return events, st.resolves

    lens = [int(x) for x in np.random.RandomState(0).randint(20, 100, size=60)]
    ev_exact, _ = run_loop(lens, exact=True)
    ev_lazy, resolves = run_loop(lens, exact=False)
    assert ev_lazy == ev_exact and len(ev_exact) > 10
    assert resolves < len(lens) // 2  # most iterations never waited for their run
