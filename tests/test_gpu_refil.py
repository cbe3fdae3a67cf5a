"""GPU parity of the REFIL path (config 5): entity env + EntityMAC rollout kernel and the
EntityAttentionRNNAgent forward against the CPU oracle (oracle/env_ref.c entity variant, oracle/refil_ref.py)
and the reference's golden vectors (tests/golden/refil_layers.npz, made by tests/golden/make_refil_golden.py).

Tolerances: env arithmetic, masks, bookkeeping and epsilon draws bit-exact; Q / hidden fp32 within 1e-4 abs.
"""
import numpy as np
import pytest
import torch

import envref
import refil_ref as RR
from helpers import entity_scheme_for, np_batch, ref_entity_envs_for, refil_args

pytestmark = pytest.mark.gpu

Q_TOL = 1e-4


def _agent(device, params=None, seed=0, **kw):
    from maleague.modules.agents import REGISTRY
    a = refil_args(**kw)
    torch.manual_seed(seed)
    ag = REGISTRY["imagine_entity_attend_rnn"](a.entity_shape + a.n_actions, a).to(device)
    if params is not None:
        ag.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in params.items()})
    return ag, a


def _params(d, prefix):
    return {k[len(prefix):]: d[k] for k in d.files if k.startswith(prefix)}


def test_agent_forward_matches_golden(device, golden):
    d = golden("refil_layers.npz")
    ag, a = _agent(device, _params(d, "agent.p."))
    ent, om, em = (torch.from_numpy(d[k]).to(device) for k in ("agent.ent", "agent.om", "agent.em"))
    h0 = torch.from_numpy(d["agent.h0"]).to(device)
    q, hs = ag((ent, om, em), h0)
    np.testing.assert_allclose(q.cpu().numpy(), d["agent.q"], atol=Q_TOL, rtol=0)
    np.testing.assert_allclose(hs.cpu().numpy(), d["agent.hs"], atol=Q_TOL, rtol=0)
    # imagination: 3 copies (plain, within, interact) with the recorded group draw
    qi, hi, (Wm, Im) = ag((ent, om, em), h0, imagine=True, groupA=torch.from_numpy(d["imagine.groupA"]).to(device))
    np.testing.assert_allclose(qi.cpu().numpy(), d["imagine.q"], atol=Q_TOL, rtol=0)
    np.testing.assert_array_equal(Wm.cpu().numpy(), d["imagine.Wmask"])
    np.testing.assert_array_equal(Im.cpu().numpy(), d["imagine.Imask"])


def _rollout(device, B=12, T=40, seed=5, eps=0.0, test_mode=True, ring=None, agent_seed=1, st=None, kmin=3, kmax=8,
             batch=None, extent=None):
    from maleague import _native
    from maleague.components.episode_batch import EpisodeBatch
    from maleague.components.batch_view import mlg_entity_batch
    from maleague.envs.entity_env import EntityEnvSpec
    from maleague.envs.teams_env import VecEnvState
    spec = EntityEnvSpec.from_env_args({"match_build_plan": "refil_8", "episode_limit": T, "seed": seed,
                                        "min_agents": kmin, "max_agents": kmax})
    ag, a = _agent(device, seed=agent_seed)
    info = spec.env_info()
    scheme, groups, pre = entity_scheme_for(info, torch)
    if st is None:
        st = VecEnvState(spec, B, device)
    if batch is None:
        batch = EpisodeBatch(scheme, groups, B, T + 1, preprocess=pre, device=device)
        if ring is not None:
            for v in batch.data.transition_data.values():
                v.fill_(7)
    mb, keep = mlg_entity_batch(batch)
    if ring is not None:
        mb.full_write = 1
    if extent is not None:
        mb.slot_extent = extent.data_ptr()
    run = torch.zeros(6 * B, dtype=torch.int32, device=device)
    ri = _native.MlgRunInfo(run[0:B].data_ptr(), run[4 * B:5 * B].data_ptr(), run[B:3 * B].data_ptr(),
                            run[3 * B:4 * B].data_ptr(), None, None)
    _native.call("mlg_refil_rollout", _native.byref(spec.to_c()), _native.byref(st.to_c()), _native.byref(ag.dims()),
                 _native.ptr(ag.packed()), _native.byref(mb), _native.byref(ri), float(eps), int(test_mode),
                 _native.stream_ptr())
    torch.cuda.synchronize()
    r = run.cpu().numpy()
    summary = {"len": r[0:B], "won": r[B:3 * B].reshape(B, 2), "draw": r[3 * B:4 * B],
               "ret": r[4 * B:5 * B].view(np.float32)}
    if extent is not None:
        _rollout.last_batch = batch
    return spec, ag, a, np_batch(batch), summary, st


@pytest.fixture(params=["v4", "v4g", "v1"])
def rollout_variant(request, monkeypatch):
    """v4: four envs per wave (refil_ro4.inc, the default; the refil_8 plan runs its static-shape instantiation);
    v4g: the same kernel's generic instantiation (MLG_REFIL_GENERIC=1); v1: the two-env kernel (MLG_REFIL_ROLLOUT=v1)."""
    monkeypatch.setenv("MLG_REFIL_ROLLOUT", "v1" if request.param == "v1" else "v4")
    if request.param == "v4g":
        monkeypatch.setenv("MLG_REFIL_GENERIC", "1")
    return request.param


def test_rollout_static_shape_equals_generic(device, monkeypatch):
    """The refil_8 static-shape instantiation of the four-env kernel (layout offsets and dims as immediates) writes
    the same bytes as its generic instantiation: 256 envs (16 workgroups), train mode, episode limit 100."""
    from maleague.envs.teams_env import VecEnvState
    B, T, seed, eps = 256, 100, 3, 0.1
    spec, ag, a, nb0, s0, _ = _rollout(device, B, T, seed, eps, test_mode=False)
    monkeypatch.setenv("MLG_REFIL_GENERIC", "1")
    *_, nb1, s1, _ = _rollout(device, B, T, seed, eps, test_mode=False, st=VecEnvState(spec, B, device))
    for k in nb0:
        np.testing.assert_array_equal(nb0[k], nb1[k], err_msg=k)
    for k in s0:
        np.testing.assert_array_equal(s0[k], s1[k], err_msg=k)


@pytest.mark.parametrize("eps,test_mode,B,T,seed", [(0.0, True, 12, 40, 5), (0.3, False, 12, 40, 5),
                                                    (0.05, False, 64, 100, 11)])
def test_rollout_teacher_forced_vs_oracle(device, rollout_variant, eps, test_mode, B, T, seed):
    """Teacher-forced: the oracle env replays the recorded actions; every greedy pick is an oracle argmax within Q_TOL,
    every epsilon draw bit-exact. The 64-env case runs config 5's episode limit (100) with partial workgroups."""
    spec, ag, a, nb, summ, _ = _rollout(device, B, T, seed, eps, test_mode)
    _teacher_check(spec, ag, a, nb, summ, B, T, seed, eps, test_mode)


def _teacher_check(spec, ag, a, nb, summ, B, T, seed, eps, test_mode, envs=None):
    """Replay the recorded actions of ``envs`` (default: all) through the oracle entity env; every greedy pick an
    oracle argmax within Q_TOL, every epsilon draw bit-exact, bookkeeping and summary exact."""
    envs = list(range(B)) if envs is None else [int(e) for e in envs]
    refs = ref_entity_envs_for(spec, B, seed=seed)
    NA, A = spec.n_agents, spec.n_actions
    p = {k: v.detach().cpu() for k, v in ag.state_dict().items()}
    qref, _ = RR.mac_forward(p, {k: torch.from_numpy(v[envs]) for k, v in nb.items()}, a)
    qref = dict(zip(envs, qref.numpy()))
    n_rand = n_greedy = 0
    for b in envs:
        r = refs[b]
        r.reset()
        L = int(summ["len"][b])
        assert 1 <= L <= T
        ret = np.float32(0)
        for t in range(L + 1):
            ent, om, em = r.entities()
            np.testing.assert_array_equal(nb["entities"][b, t], ent, err_msg=f"entities b={b} t={t}")
            np.testing.assert_array_equal(nb["obs_mask"][b, t], om, err_msg=f"obs_mask b={b} t={t}")
            np.testing.assert_array_equal(nb["entity_mask"][b, t], em)
            av = r.avail()
            np.testing.assert_array_equal(nb["avail_actions"][b, t], av)
            assert nb["filled"][b, t, 0] == 1
            acts = nb["actions"][b, t, :, 0]
            for n in range(NA):
                key = envref.env_key(seed, b)
                coin = not test_mode and eps > 0 and envref.u01(envref.rng(key, envref.ctr(r.cur_episode, t, 2, n))) < eps
                if coin:
                    want = envref.random_available(av[n], envref.rng(key, envref.ctr(r.cur_episode, t, 3, n)))
                    assert acts[n] == want
                    n_rand += 1
                else:
                    qm = np.where(av[n] != 0, qref[b][t, n], -np.inf)
                    assert av[n, acts[n]] != 0 and qm[acts[n]] >= qm.max() - Q_TOL, (b, t, n)
                    n_greedy += 1
            oh = np.zeros((NA, A), np.float32)
            oh[np.arange(NA), acts] = 1
            np.testing.assert_array_equal(nb["actions_onehot"][b, t], oh)
            if t < L:
                rew, done, info = r.step(acts)
                assert nb["reward"][b, t, 0] == np.float32(rew[0])
                assert nb["terminated"][b, t, 0] == int(done)
                assert done == (t == L - 1)
                ret += np.float32(rew[0])
        assert summ["won"][b, 0] == int(info["battle_won"][0]) and summ["won"][b, 1] == int(info["battle_won"][1])
        assert summ["draw"][b] == int(info["draw"])
        assert abs(summ["ret"][b] - ret) <= 1e-3
        assert nb["filled"][b, L + 1:].sum() == 0 and nb["reward"][b, L:].sum() == 0
    assert n_greedy > 0 and (test_mode or n_rand > 0)
    return n_greedy, n_rand


def test_rollout_config5_full_shape(device):
    """BASELINE config 5 at its launch shape (4096 envs, episode limit 100, 3-8 agents per env, train mode at the
    steady-state epsilon 0.05; 256 workgroups of the four-env kernel in one round): size-independent invariants,
    determinism (same episode counters -> bit-identical batch and summary), and 64 envs spread over the launch
    teacher-forced against the oracle env + oracle EntityMAC."""
    from maleague.envs.teams_env import VecEnvState
    B, T, seed, eps = 4096, 100, 0, 0.05
    spec, ag, a, nb, summ, st = _rollout(device, B, T, seed, eps, test_mode=False)
    L = summ["len"]
    assert (L >= 1).all() and (L <= T).all()
    assert nb["filled"].sum() == (L + 1).sum() and nb["terminated"].sum() == B
    filled = nb["filled"][:, :, 0] == 1
    assert (nb["actions_onehot"].sum(-1)[filled] == 1).all()
    av_taken = np.take_along_axis(nb["avail_actions"], nb["actions"].astype(np.int64), axis=-1)[..., 0]
    assert (av_taken[filled] == 1).all(), "every recorded action is available"
    assert (np.mod(nb["reward"] * 16, 1) == 0).all()
    # agents per env: the active slots of the policy team are the first k entities, k in [3, 8]
    alive0 = (nb["entity_mask"][:, 0, :8] == 0).sum(-1)
    assert alive0.min() >= 3 and alive0.max() <= 8 and len(np.unique(alive0)) == 6
    # determinism
    spec2, ag2, a2, nb2, summ2, _ = _rollout(device, B, T, seed, eps, test_mode=False, st=VecEnvState(spec, B, device))
    for k in nb:
        np.testing.assert_array_equal(nb[k], nb2[k], err_msg=k)
    for k in summ:
        np.testing.assert_array_equal(summ[k], summ2[k], err_msg=k)
    sub = np.linspace(0, B - 1, 64).astype(int)
    n_greedy, n_rand = _teacher_check(spec, ag, a, nb, summ, B, T, seed, eps, False, envs=sub)
    assert n_greedy > 1000 and n_rand > 0


def test_rollout_ring_full_write_equals_zeroed(device, rollout_variant):
    """full-write mode writes every byte of the slots (garbage-filled here): identical to the zeroed batch."""
    *_, nb0, s0, st = _rollout(device, B=10, T=30, seed=9, eps=0.2, test_mode=False)
    # same env state as the first run started from: a fresh state advanced by nothing
    *_, nb1, s1, _ = _rollout(device, B=10, T=30, seed=9, eps=0.2, test_mode=False, ring=True)
    for k in nb0:
        np.testing.assert_array_equal(nb0[k], nb1[k], err_msg=k)
    np.testing.assert_array_equal(s0["len"], s1["len"])


def test_rollout_full_write_slot_extents(device, rollout_variant):
    """full-write mode with slot extents (MlgEntityBatch.slot_extent): one batch rewritten by successive runs of
    different episodes; each run zeroes only the rows past its episodes' ends that the previous episode in the slot
    wrote, records L + 1, and the batch equals a zero-initialised one every time."""
    B, T = 10, 30
    ext = torch.full((B,), T + 1, dtype=torch.int32, device=device)  # rows unknown: a fresh garbage-filled batch
    batch = None
    for it, (seed, eps) in enumerate([(9, 0.2), (3, 0.6), (9, 0.0), (5, 0.3)]):
        *_, nb0, s0, _ = _rollout(device, B=B, T=T, seed=seed, eps=eps, test_mode=False)  # zero-initialised
        *_, nb1, s1, _ = _rollout(device, B=B, T=T, seed=seed, eps=eps, test_mode=False, ring=True, batch=batch,
                                  extent=ext)
        batch = _rollout.last_batch
        for k in nb0:
            np.testing.assert_array_equal(nb0[k], nb1[k], err_msg=f"{it} {k}")
        np.testing.assert_array_equal(ext.cpu().numpy(), s1["len"] + 1)


def test_rollout_fixed_team_sizes(device, rollout_variant):
    """k = 8 (full teams) and k = 3 (smallest): absent slots masked, padded agents only no-op."""
    for k in (3, 8):
        spec, ag, a, nb, summ, _ = _rollout(device, B=6, T=25, seed=2, kmin=k, kmax=k)
        em = nb["entity_mask"][:, 0]
        assert (em[:, :k] == 0).all() and (em[:, k:8] == 1).all() and (em[:, 8:8 + k] == 0).all()
        if k < 8:
            av = nb["avail_actions"][:, 0, k:]
            assert (av[..., 0] == 1).all() and (av[..., 1:] == 0).all()
            assert (nb["actions"][:, 0, k:, 0] == 0).all()


@pytest.mark.parametrize("tag,nq", [("na", 8), ("ne", 16)])
def test_attention_layer_forward_backward_golden(device, golden, tag, nq):
    """EntityAttentionLayer fwd + bwd (mlg_refil_attention) vs the reference's vectors (attention.py:24-79)."""
    from maleague import _native
    d = golden("refil_layers.npz")
    t = lambda k, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(d[k])).to(device=device, dtype=dt)  # noqa
    w_in, w_out, b_out = t("attn.p.in_trans.weight"), t("attn.p.out_trans.weight"), t("attn.p.out_trans.bias")
    x = t("attn.x")
    bs, ne, _ = x.shape
    pre = t("attn.pre", torch.uint8)[:, :nq].contiguous()
    post = t("attn.em", torch.uint8)[:, :nq].contiguous()
    gy = t(f"attn.{tag}.g")
    y = torch.empty(bs, nq, 64, device=device)
    dx = torch.empty_like(x)
    dwi, dwo, dbo = torch.zeros_like(w_in), torch.zeros_like(w_out), torch.zeros_like(b_out)
    P = _native.ptr
    _native.call("mlg_refil_attention", P(w_in), P(w_out), P(b_out), P(x), P(pre), P(post), bs, ne, nq, 4, P(y), P(gy),
                 P(dx), P(dwi), P(dwo), P(dbo), _native.stream_ptr())
    np.testing.assert_allclose(y.cpu().numpy(), d[f"attn.{tag}.y"], atol=Q_TOL, rtol=0)
    np.testing.assert_allclose(dx.cpu().numpy(), d[f"attn.{tag}.dx"], atol=Q_TOL, rtol=0)
    np.testing.assert_allclose(dwi.cpu().numpy(), d[f"attn.{tag}.d.in_trans.weight"], atol=Q_TOL, rtol=1e-4)
    np.testing.assert_allclose(dwo.cpu().numpy(), d[f"attn.{tag}.d.out_trans.weight"], atol=Q_TOL, rtol=1e-4)
    np.testing.assert_allclose(dbo.cpu().numpy(), d[f"attn.{tag}.d.out_trans.bias"], atol=Q_TOL, rtol=1e-4)


@pytest.mark.parametrize("tag", ["abs", "soft"])
def test_flex_qmixer_forward_golden(device, golden, tag):
    """FlexQMixer.forward plain and with imagine groups (flex_qmix.py:73-117) vs the reference's vectors."""
    from maleague.modules.mixers import FlexQMixer
    d = golden("refil_layers.npz")
    a = refil_args(softmax_mixing_weights=tag == "soft")
    m = FlexQMixer(a).to(device)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in _params(d, f"mixer.{tag}.p.").items()})
    g = lambda k: torch.from_numpy(d[f"mixer.{tag}.{k}"]).to(device)  # noqa: E731
    y = m(g("qs"), (g("ent"), g("em")))
    np.testing.assert_allclose(y.cpu().numpy(), d[f"mixer.{tag}.y"], atol=Q_TOL, rtol=1e-5)
    y2 = m(g("qs2"), (g("ent"), g("em")), imagine_groups=(g("wm"), g("im")))
    np.testing.assert_allclose(y2.cpu().numpy(), d[f"mixer.{tag}.y2"], atol=Q_TOL, rtol=1e-5)
