"""GPU parity of the env / agent / rollout kernels (libmaleague.so, gfx950) against the CPU oracle
(oracle/env_ref.c, oracle/learner_ref.py, oracle/stepper_ref.py) and the reference's golden vectors.

Tolerances: env arithmetic, masks, bookkeeping and argmax/epsilon indices are bit-exact; Q-values and
hidden states are fp32 and checked within 1e-4 abs (north_star) -- in practice ~1e-6.
"""
import numpy as np
import pytest
import torch

import envref
import learner_ref as LR
from helpers import assert_near_tie_divergence, np_batch, qmix_args, ref_envs_for, scheme_for

pytestmark = pytest.mark.gpu

Q_TOL = 1e-4
# the measured number of v7 episodes (of 100) that diverge from v2 at a near-tie argmax flip,
# per plan (static and runtime shapes), pinned with a small margin (was a blanket B // 10)
V7_MAX_DIVERGING = {"medium_1h_4t": 2, "medium": 2, "small": 2}  # measured 0 / 0 / 0 (both shapes, r05)


def _mk_env(device, plan, B, episode_limit=60, seed=3, stochastic=True):
    from maleague.envs.teams_env import TeamsEnvSpec, VecEnvState
    spec = TeamsEnvSpec.from_env_args({"match_build_plan": plan, "grid_size": 20, "stochastic_spawns": stochastic,
                                       "episode_limit": episode_limit, "seed": seed})
    return spec, VecEnvState(spec, B, device)


@pytest.mark.parametrize("plan,stochastic", [("small", True), ("medium_1h_4t", True), ("medium_1h_2t_2a_melee", True),
                                             ("medium_1h_4a", False), ("large", True)])
def test_env_kernels_bit_exact(device, plan, stochastic):
    from maleague import _native
    B, T = 24, 50
    spec, st = _mk_env(device, plan, B, episode_limit=T, seed=7, stochastic=stochastic)
    cspec = spec.to_c()
    refs = ref_envs_for(spec, B, seed=7)
    U, N, A = spec.U, spec.n_agents, spec.n_actions
    obs = torch.zeros(B, N, 8 * U, device=device)
    state = torch.zeros(B, 6 * U, device=device)
    avail = torch.zeros(B, N, A, dtype=torch.int32, device=device)
    rew = torch.zeros(B, spec.n_policy_teams, device=device)
    done = torch.zeros(B, dtype=torch.int32, device=device)
    won = torch.zeros(B, 2, dtype=torch.int32, device=device)
    draw = torch.zeros(B, dtype=torch.int32, device=device)
    _native.call("mlg_env_reset", _native.byref(cspec), _native.byref(st.to_c()), _native.stream_ptr())
    for r in refs:
        r.reset()
    rng = np.random.RandomState(0)
    for t in range(T):
        _native.call("mlg_env_observe", _native.byref(cspec), _native.byref(st.to_c()), _native.ptr(obs),
                     _native.ptr(state), _native.ptr(avail), _native.stream_ptr())
        np.testing.assert_array_equal(st.x.cpu().numpy(), np.stack([r.x for r in refs]))
        np.testing.assert_array_equal(st.y.cpu().numpy(), np.stack([r.y for r in refs]))
        np.testing.assert_array_equal(st.hp.cpu().numpy(), np.stack([r.hp for r in refs]))
        np.testing.assert_array_equal(obs.cpu().numpy(), np.stack([r.obs() for r in refs]))
        np.testing.assert_array_equal(state.cpu().numpy(), np.stack([r.state() for r in refs]))
        av = avail.cpu().numpy()
        np.testing.assert_array_equal(av, np.stack([r.avail() for r in refs]))
        acts = np.zeros((B, N), np.int64)
        for b in range(B):
            for n in range(N):
                ok = np.nonzero(av[b, n])[0]
                acts[b, n] = rng.randint(A + 3) - 1 if rng.rand() < 0.1 else rng.choice(ok)  # some invalid -> noop
        a_t = torch.from_numpy(acts).to(device)
        _native.call("mlg_env_step", _native.byref(cspec), _native.byref(st.to_c()), _native.ptr(a_t), _native.ptr(rew),
                     _native.ptr(done), _native.ptr(won), _native.ptr(draw), _native.stream_ptr())
        exp = [r.step(acts[b]) for b, r in enumerate(refs)]
        np.testing.assert_array_equal(rew.cpu().numpy(), np.array([e[0] for e in exp], np.float32))
        np.testing.assert_array_equal(done.cpu().numpy(), np.array([e[1] for e in exp], np.int32))
        np.testing.assert_array_equal(won.cpu().numpy(), np.array([e[2]["battle_won"] for e in exp], np.int32))
        np.testing.assert_array_equal(draw.cpu().numpy(), np.array([e[2]["draw"] for e in exp], np.int32))


def test_agent_forward_golden(device, golden):
    from maleague.modules.agents.drqn_agent import DRQNAgentNetwork
    d = golden("drqn_step.npz")
    args = qmix_args(n_agents=5, n_actions=15)
    agent = DRQNAgentNetwork(100, args)
    agent.load_state_dict({k[2:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith("p.")})
    q, h = agent(torch.from_numpy(d["inputs"]).to(device), torch.from_numpy(d["hidden"]).to(device))
    np.testing.assert_allclose(q.cpu().numpy(), d["q"], atol=Q_TOL, rtol=0)
    np.testing.assert_allclose(h.cpu().numpy(), d["h"], atol=Q_TOL, rtol=0)
    # ragged row count (not a multiple of the 16-row tile)
    q2, h2 = agent(torch.from_numpy(d["inputs"][:27]).to(device), torch.from_numpy(d["hidden"][:27]).to(device))
    np.testing.assert_allclose(q2.cpu().numpy(), d["q"][:27], atol=Q_TOL, rtol=0)


def _golden_batch(d, device):
    from maleague.components.episode_batch import EpisodeBatch
    b = LR.batch_from_npz(d)
    B, T, N, _ = b["obs"].shape
    A = b["avail_actions"].shape[-1]
    env_info = {"state_shape": b["state"].shape[-1], "obs_shape": b["obs"].shape[-1], "n_actions": A, "n_agents": N}
    scheme, groups, preprocess = scheme_for(env_info, torch)
    eb = EpisodeBatch(scheme, groups, B, T, preprocess=preprocess, device=device)
    for k, v in b.items():
        eb.data.transition_data[k].copy_(v)
    return eb


def test_mac_forward_golden(device, golden):
    from maleague.controllers import BasicMAC
    d = golden("mac_forward.npz")
    eb = _golden_batch(d, device)
    mac = BasicMAC(eb.scheme, eb.groups, qmix_args())
    mac.load_state_dict({k[2:]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith("p.")})
    mac.init_hidden(eb.batch_size)
    for t in range(eb.max_seq_length):
        q = mac.forward(eb, t)
        np.testing.assert_allclose(q.cpu().numpy(), d["q"][t], atol=Q_TOL, rtol=0, err_msg=f"t={t}")


def test_select_actions_golden(device, golden):
    from maleague.components.action_selectors import EpsilonGreedyActionSelector
    d = golden("eps_greedy.npz")
    sel = EpsilonGreedyActionSelector(qmix_args())
    a, g = sel.select(torch.from_numpy(d["q"]).to(device), torch.from_numpy(d["avail"]).to(device), 0, test_mode=True)
    np.testing.assert_array_equal(a.cpu().numpy(), d["actions"])
    np.testing.assert_array_equal(g.cpu().numpy(), d["is_greedy"])


def test_select_actions_epsilon_stream(device):
    from maleague import _native
    rng = np.random.RandomState(1)
    B, N, A = 40, 5, 15
    q = rng.randn(B, N, A).astype(np.float32)
    av = (rng.rand(B, N, A) < 0.4).astype(np.int32)
    av[..., 4] = 1
    keys = np.array([(9 << 32) + b for b in range(B)], np.uint64)
    eps_ = np.arange(B, dtype=np.int64) % 3
    acts = torch.zeros(B, N, dtype=torch.int64, device=device)
    greedy = torch.zeros(B, N, dtype=torch.int64, device=device)
    qd, ad = torch.from_numpy(q).to(device), torch.from_numpy(av).to(device)
    kd = torch.from_numpy(keys.view(np.int64)).to(device)
    ed = torch.from_numpy(eps_.astype(np.int32)).to(device)
    _native.call("mlg_select_actions", _native.ptr(qd), _native.ptr(ad), B * N, A, N, _native.ptr(kd), _native.ptr(ed),
                 7, 0.6, _native.ptr(acts), _native.ptr(greedy), _native.stream_ptr())
    exp, exp_g = LR.eps_select(torch.from_numpy(q), torch.from_numpy(av), 0.6, [int(k) for k in keys],
                               [int(e) for e in eps_], 7)
    np.testing.assert_array_equal(acts.cpu().numpy(), exp)
    np.testing.assert_array_equal(greedy.cpu().numpy(), exp_g)
    assert 0 < (exp_g == 0).sum() < B * N


def _build_stepper(device, plan="medium_1h_4t", B=48, episode_limit=40, seed=5, **kw):
    from maleague.components.episode_batch import EpisodeBatch
    from maleague.controllers import BasicMAC
    from maleague.custom_logging import MainLogger
    from maleague.steppers import ParallelStepper
    args = qmix_args(batch_size_run=B, seed=seed, env_args={"match_build_plan": plan, "grid_size": 20,
                                                            "stochastic_spawns": True, "episode_limit": episode_limit},
                     **kw)
    stepper = ParallelStepper(args, MainLogger())
    info = stepper.get_env_info()
    args.n_agents, args.n_actions, args.state_shape = info["n_agents"], info["n_actions"], info["state_shape"]
    scheme, groups, preprocess = scheme_for(info, torch)
    proto = EpisodeBatch(scheme, groups, 1, 2, preprocess=preprocess, device=device)
    torch.manual_seed(seed)
    mac = BasicMAC(proto.scheme, groups, args)
    stepper.initialize(scheme, groups, preprocess, mac)
    return stepper, mac, args


def _check_run(stepper, mac, args, batch, infos, episode, test_mode, eps, envs=None):
    """Teacher-forced env replay + oracle agent check of a run; ``envs``: the env indices to check (all by
    default; a subset for the 4096-env headline shape)."""
    spec = stepper.spec
    B, N, A, T1 = stepper.batch_size, spec.n_agents, spec.n_actions, stepper.episode_limit + 1
    sub = list(range(B)) if envs is None else [int(e) for e in envs]
    nb = np_batch(batch)
    ep_len = stepper.last_run["ep_len"].numpy()
    rets = stepper.last_run["returns"].numpy()
    assert (ep_len >= 1).all() and (ep_len <= stepper.episode_limit).all()
    assert stepper.t == ep_len.max()
    # --- env side, teacher forced: replay the recorded actions through the C oracle ---
    refs = ref_envs_for(spec, B, seed=args.seed)
    for b in sub:
        r = refs[b]
        r.episode = episode
        r.reset()
        L = int(ep_len[b])
        np.testing.assert_array_equal(nb["obs"][b, 0], r.obs())
        np.testing.assert_array_equal(nb["state"][b, 0], r.state())
        np.testing.assert_array_equal(nb["avail_actions"][b, 0], r.avail())
        ret = 0.0
        for t in range(L):
            rew, done, info = r.step(nb["actions"][b, t, :, 0])
            ret += rew[0]
            assert nb["reward"][b, t, 0] == np.float32(rew[0])
            assert nb["terminated"][b, t, 0] == int(done) and done == (t == L - 1)
            np.testing.assert_array_equal(nb["obs"][b, t + 1], r.obs())
            np.testing.assert_array_equal(nb["state"][b, t + 1], r.state())
            np.testing.assert_array_equal(nb["avail_actions"][b, t + 1], r.avail())
        assert rets[b] == np.float32(ret)
        np.testing.assert_array_equal(nb["filled"][b, :, 0], (np.arange(T1) <= L).astype(np.int64))
        # actions recorded for t = 0..L (the final one after termination), zero beyond
        assert (nb["actions"][b, L + 1:] == 0).all() and (nb["actions_onehot"][b, L + 1:] == 0).all()
        oh = np.zeros((L + 1, N, A), np.float32)
        oh[np.arange(L + 1)[:, None], np.arange(N)[None, :], nb["actions"][b, :L + 1, :, 0]] = 1
        np.testing.assert_array_equal(nb["actions_onehot"][b, :L + 1], oh)
        assert (nb["reward"][b, L:] == 0).all() and (nb["terminated"][b, L:] == 0).all()
    # env_infos in order of termination
    order = sorted(range(B), key=lambda i: (int(ep_len[i]), i))
    assert len(infos) == B
    # --- agent side: oracle Q on the recorded batch; greedy / epsilon picks bit-exact ---
    params = {k: v.detach().cpu() for k, v in mac.agent.state_dict().items()}
    tb = {k: torch.from_numpy(v[sub]) for k, v in nb.items()}
    Tm = int(ep_len[sub].max()) + 1
    with torch.no_grad():
        q, _ = LR.mac_unroll(params, tb, N, T=Tm)
    q = dict(zip(sub, q.numpy()))
    n_checked = n_random = 0
    for b in sub:
        for t in range(int(ep_len[b]) + 1):
            for n in range(N):
                a = int(nb["actions"][b, t, n, 0])
                av = nb["avail_actions"][b, t, n]
                if not test_mode and eps > 0:
                    key = envref.env_key(args.seed, b)
                    r1 = envref.rng(key, envref.ctr(episode, t, 2, n))
                    if envref.u01(r1) < np.float32(eps):
                        r2 = envref.rng(key, envref.ctr(episode, t, 3, n))
                        assert a == envref.random_available(av.tolist(), r2)
                        n_random += 1
                        continue
                m = np.where(av == 0, -np.inf, q[b][t, n])
                g = int(np.argmax(m))
                srt = np.sort(m)
                if srt[-1] - srt[-2] > Q_TOL:
                    assert a == g, (b, t, n, a, g)
                else:  # near-tie within fp32 tolerance: chosen must be (numerically) a max
                    assert m[a] >= srt[-1] - Q_TOL
                n_checked += 1
    assert n_checked > 0
    if not test_mode and eps > 0.2:
        assert n_random > 0
    return order


@pytest.mark.parametrize("plan", ["medium_1h_4t", "small", "medium_1h_2t_2a"])
def test_rollout_teacher_forced_parity(device, plan):
    stepper, mac, args = _build_stepper(device, plan=plan, B=48, episode_limit=40)
    batch, infos = stepper.run(test_mode=True)
    _check_run(stepper, mac, args, batch, infos, episode=0, test_mode=True, eps=0.0)
    assert stepper.t_env == 0
    stepper.t_env = 25000  # epsilon = 1 - 0.95 * 0.5 = 0.525
    eps = max(0.05, 1.0 - 0.95 / 50000 * 25000)
    batch, infos = stepper.run(test_mode=False)
    _check_run(stepper, mac, args, batch, infos, episode=1, test_mode=False, eps=eps)
    assert stepper.t_env == 25000 + int(stepper.last_run["ep_len"].sum())


def test_rollout_headline_config_properties(device):
    """BASELINE config 2 shape (5v5, 4096 envs, episode_limit 100): size-independent invariants + determinism."""
    stepper, mac, args = _build_stepper(device, plan="medium_1h_4t", B=4096, episode_limit=100, seed=0)
    stepper.t_env = 10 ** 6  # steady-state epsilon 0.05
    batch, infos = stepper.run(test_mode=False)
    nb = np_batch(batch)
    L = stepper.last_run["ep_len"].numpy()
    assert nb["filled"].sum() == (L + 1).sum()
    assert nb["terminated"].sum() == 4096
    assert (nb["actions_onehot"].sum(-1)[nb["filled"][:, :, 0] == 1] == 1).all()
    assert (np.mod(nb["reward"] * 16, 1) == 0).all()
    av_taken = np.take_along_axis(nb["avail_actions"], nb["actions"].astype(np.int64), axis=-1)[..., 0]
    assert (av_taken[nb["filled"][:, :, 0] == 1] == 1).all(), "every recorded action is available"
    # determinism: same episode counters -> bitwise identical batch
    from maleague.envs.teams_env import VecEnvState
    stepper.envs = VecEnvState(stepper.spec, 4096, device)
    stepper.t_env = 10 ** 6
    b1, _ = stepper.run(test_mode=False)
    stepper.envs = VecEnvState(stepper.spec, 4096, device)
    stepper.t_env = 10 ** 6
    b2, _ = stepper.run(test_mode=False)
    for k in b1.data.transition_data:
        assert torch.equal(b1[k], b2[k]), k
    # teacher-forced spot check of 64 envs of the big run
    sub = [int(i) for i in np.linspace(0, 4095, 64)]
    refs = ref_envs_for(stepper.spec, 4096, seed=0)
    nb = np_batch(b1)
    L = stepper.last_run["ep_len"].numpy()
    for b in sub:
        r = refs[b]
        r.episode = 0
        r.reset()
        for t in range(int(L[b])):
            rew, done, _ = r.step(nb["actions"][b, t, :, 0])
            assert nb["reward"][b, t, 0] == np.float32(rew[0])
            np.testing.assert_array_equal(nb["obs"][b, t + 1], r.obs())


def test_rollout_headline_config_agent_parity(device):
    """BASELINE config 2 at its full shape (5v5, 4096 envs, episode_limit 100, train mode at the steady-state
    epsilon 0.05, the v7 kernel): 64 envs spread over the launch replayed through the C env and the fp32 oracle
    DRQN -- every epsilon draw bit-exact vs the oracle counter RNG, every greedy pick the oracle's argmax (near
    ties within Q_TOL), env transitions bit-exact."""
    stepper, mac, args = _build_stepper(device, plan="medium_1h_4t", B=4096, episode_limit=100, seed=0)
    stepper.t_env = 10 ** 6
    eps = max(0.05, 1.0 - 0.95 / 50000 * 10 ** 6)
    batch, infos = stepper.run(test_mode=False)
    sub = np.linspace(0, 4095, 64).astype(int)
    _check_run(stepper, mac, args, batch, infos, episode=0, test_mode=False, eps=eps, envs=sub)


def test_stepper_summary_ring_runahead_matches_resolved(device):
    """the host runs up to _HOST_RING train-mode runs ahead of the device (run summaries written by the
    kernel into a ring of pinned buffers, t_env unresolved). Ten runs across the end of the epsilon anneal, never
    reading t_env, must equal the same runs stepped with a resolve after each run: same epsilon per run (=
    schedule.eval of the exact t_env), same episodes, same final t_env; the ring fills up (oldest run resolved
    first) once the schedule is flat."""
    from maleague.envs.teams_env import VecEnvState
    runs = {}
    for mode in ("ahead", "resolved"):
        stepper, mac, args = _build_stepper(device, plan="medium_1h_4t", B=64, episode_limit=60, seed=4,
                                            epsilon_anneal_time=6000)
        stepper.envs = VecEnvState(stepper.spec, 64, device)
        stepper.t_env = 0
        eps, batches, pend, exact = [], [], [], []
        for _ in range(10):
            b, infos = stepper.run(test_mode=False)
            eps.append(float(mac.action_selector.epsilon))
            pend.append(len(stepper._pendings))
            batches.append({k: b[k].clone() for k in b.data.transition_data})
            if mode == "resolved":
                exact.append(stepper.t_env)
        runs[mode] = (eps, batches, pend, stepper.t_env, exact, [bool(i["battle_won"][0]) for i in infos])
    ea, ba, pa, ta, _, wa = runs["ahead"]
    er, br, _, tr, exact, wr = runs["resolved"]
    assert ta == tr and wa == wr
    assert ea == er
    sched = _build_stepper(device, B=64, epsilon_anneal_time=6000)[1].action_selector.schedule
    t_before = [0] + exact[:-1]
    assert ea == [float(sched.eval(t)) for t in t_before]
    assert ea[0] > ea[-1] == 0.05 and ea[1] > 0.05, ea  # annealing at first, flat at the end
    assert max(pa) == stepper._HOST_RING, pa  # ring full: the oldest run was resolved to make room
    for i, (x, y) in enumerate(zip(ba, br)):
        for k in x:
            assert torch.equal(x[k], y[k]), (i, k)


@pytest.mark.parametrize("kernel", ["v7", "v2", "v1"])
def test_rollout_ring_mode_zero_copy_insert(device, kernel, monkeypatch):
    """Train-mode rollouts written straight into the replay ring (full-write mode, wrap-around, garbage in the
    slots beforehand) equal the ordinary zero-initialised EpisodeBatch bit for bit, and the buffer indices
    advance exactly like ReplayBuffer.insert_episode_batch."""
    from maleague.components.replay_buffer import ReplayBuffer
    from maleague.envs.teams_env import VecEnvState
    monkeypatch.setenv("MLG_ROLLOUT_KERNEL", kernel)
    stepper, mac, args = _build_stepper(device, plan="medium_1h_4t", B=48, episode_limit=30, seed=2)
    info = stepper.get_env_info()
    scheme, groups, preprocess = scheme_for(info, torch)
    ring = ReplayBuffer(scheme, groups, 100, 31, preprocess=preprocess, device=device)
    ref = ReplayBuffer(scheme, groups, 100, 31, preprocess=preprocess, device=device)
    for v in ring.data.transition_data.values():
        v.fill_(7)
    stepper.t_env = 20000
    for it in range(4):  # slots 0-47, 48-95, 96-43 (wraps), 44-91
        st0 = VecEnvState(stepper.spec, 48, device)
        st0.episode.fill_(it)
        stepper.envs = st0
        stepper._ring = None
        b_plain, _ = stepper.run(test_mode=False)
        stepper.t_env -= int(stepper.last_run["ep_len"].sum())
        st1 = VecEnvState(stepper.spec, 48, device)
        st1.episode.fill_(it)
        stepper.envs = st1
        assert stepper.attach_replay(ring)
        b_ring, _ = stepper.run(test_mode=False)
        for k in b_plain.data.transition_data:
            assert torch.equal(b_plain[k], b_ring[k]), (it, k)
        ring.insert_episode_batch(b_ring)
        ref.insert_episode_batch(b_plain)
        assert (ring.buffer_index, ring.episodes_in_buffer) == (ref.buffer_index, ref.episodes_in_buffer)
        # slot extents (MlgBatch.slot_extent): the run's slots now hold rows [0, L] of their episodes
        slots = (torch.arange(48) + b_ring.slot0) % 100
        want = (stepper.last_run["ep_len"] + 1).to(torch.int32)
        assert torch.equal(ring.slot_extent.cpu()[slots], want), (it, kernel)
    for k in ref.data.transition_data:
        n = ref.episodes_in_buffer
        assert torch.equal(ring[k][:n], ref[k][:n]), k


@pytest.mark.parametrize("kernel", ["v2"])
@pytest.mark.parametrize("plan", ["medium_1h_4t", "small", "medium_1h_2t_2a", "medium"])
def test_rollout_v2_equals_v1(device, plan, kernel, monkeypatch):
    """The chunk-split, compacted headline kernel (v2) and the generic per-tile kernel (v1) compute in the same
    arithmetic order: the whole batch and the run summary must be bit-identical."""
    from maleague.envs.teams_env import VecEnvState
    stepper, mac, args = _build_stepper(device, plan=plan, B=100, episode_limit=60, seed=3)
    out = {}
    for k in ("v1", kernel):
        monkeypatch.setenv("MLG_ROLLOUT_KERNEL", k)
        stepper.envs = VecEnvState(stepper.spec, 100, device)
        stepper.t_env = 30000
        b, _ = stepper.run(test_mode=False)
        out[k] = ({kk: b[kk].clone() for kk in b.data.transition_data},
                  {kk: v.clone() for kk, v in stepper.last_run.items() if torch.is_tensor(v)})
    for kk, v in out["v1"][0].items():
        assert torch.equal(v, out[kernel][0][kk]), kk
    for kk, v in out["v1"][1].items():
        assert torch.equal(v, out[kernel][1][kk]), kk


def test_rollout_second_run_before_insert_leaves_ring_episodes(device):
    """A second train-mode run before insert_episode_batch goes to a fresh batch: the first run's episodes,
    written in place into the ring, are not overwritten (the reference leaves the buffer untouched until insert)."""
    from maleague.components.replay_buffer import ReplayBuffer, RingEpisodeBatch
    stepper, mac, args = _build_stepper(device, plan="medium_1h_4t", B=48, episode_limit=30, seed=2)
    info = stepper.get_env_info()
    scheme, groups, preprocess = scheme_for(info, torch)
    ring = ReplayBuffer(scheme, groups, 100, 31, preprocess=preprocess, device=device)
    assert stepper.attach_replay(ring)
    stepper.t_env = 20000
    b1, _ = stepper.run(test_mode=False)
    snap = {k: v.clone() for k, v in b1.data.transition_data.items()}
    b2, _ = stepper.run(test_mode=False)
    assert isinstance(b1, RingEpisodeBatch) and not isinstance(b2, RingEpisodeBatch)
    for k, v in snap.items():
        assert torch.equal(b1[k], v), k
    assert not torch.equal(b1["actions"], b2["actions"])
    ring.insert_episode_batch(b1)
    ring.insert_episode_batch(b2)
    for k, v in snap.items():
        assert torch.equal(ring[k][:48], v), k
        assert torch.equal(ring[k][48:96], b2[k]), k


@pytest.mark.parametrize("generic", [False, True])
@pytest.mark.parametrize("plan", ["medium_1h_4t", "medium", "small"])
def test_rollout_v7_split_bf16_gru_matches_fp32(device, plan, generic, monkeypatch):
    """v7: the GRU products run on the bf16 matrix cores as split-bf16 fp32 emulation (three bf16 pieces per
    operand, six partial products, fp32 accumulation). Along v7's own recorded trajectory (test mode, epsilon 0)
    the fp32 oracle DRQN (oracle/learner_ref.py, drqn_agent.py:29-35) must rate every recorded action as an
    available argmax up to a 1e-5 tie, and v7 must reproduce v2's episodes bit for bit except where a near-tie
    of the Q values flips an argmax (env transitions of v7 are the v2 env code). generic: the runtime-shape kernel
    instead of the compile-time-shape instantiation (5v5 / 3v3 plans)."""
    from maleague.envs.teams_env import VecEnvState
    if generic:
        monkeypatch.setenv("MLG_ROLLOUT_GENERIC", "1")
    B, TL = 100, 60
    stepper, mac, args = _build_stepper(device, plan=plan, B=B, episode_limit=TL, seed=3)
    out = {}
    for k in ("v2", "v7"):
        monkeypatch.setenv("MLG_ROLLOUT_KERNEL", k)
        stepper.envs = VecEnvState(stepper.spec, B, device)
        b, _ = stepper.run(test_mode=True)
        out[k] = (np_batch(b), stepper.last_run["ep_len"].numpy().copy())
    nb, L = out["v7"]
    tb = {kk: torch.from_numpy(v) for kk, v in nb.items()}
    p = {kk: v.detach().cpu() for kk, v in mac.agent.state_dict().items()}
    q, _ = LR.mac_unroll(p, tb, args.n_agents, T=TL + 1)
    q = q.numpy()
    av = nb["avail_actions"].astype(bool)
    worst = 0.0
    for b_ in range(B):
        for t in range(int(L[b_]) + 1):  # every step incl. the final action after termination
            qm = np.where(av[b_, t], q[b_, t], -np.inf)
            best = qm.max(axis=-1)
            chosen = np.take_along_axis(qm, nb["actions"][b_, t], axis=-1)[:, 0]
            assert np.isfinite(chosen).all(), (b_, t)  # chosen action available
            worst = max(worst, float((best - chosen).max()))
    assert worst <= 1e-5, worst
    # episodes that differ from v2's must diverge at a near-tie flip of an argmax, not anywhere
    n_diff = assert_near_tie_divergence([out["v2"][0]], [nb], [q], B)
    print(f"v7 vs v2 [{plan}, generic={generic}]: {n_diff} of {B} episodes diverge (near-tie flips)")
    assert n_diff <= V7_MAX_DIVERGING[plan], (plan, generic, n_diff)
