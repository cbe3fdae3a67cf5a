"""GPU parity of REFILLearner.train (mlg_refil_train, config 5) against the reference's golden vectors (two
consecutive REFILLearner.train calls, tests/golden/refil_learner.npz) and against the CPU oracle
(oracle/refil_ref.py) on episodes produced by the HIP REFIL rollout.

Tolerances (fp32, different summation orders): stats rtol 2e-4; parameters after RMSprop atol 2e-5 (RMSprop's
first steps move weights by ~lr * sign(g) * const, so this checks sign-level gradient agreement everywhere and
the magnitudes through the second step).
"""
import numpy as np
import pytest
import torch

import refil_ref as RR
from helpers import entity_scheme_for, refil_args

pytestmark = pytest.mark.gpu


class _Log:
    def __init__(self):
        self.stats = {}

    def log_stat(self, k, v, t):
        self.stats[k] = v

    def info(self, *a):
        pass


def _batch_from(arrs, device, NE=16, ED=8, NA=8, A=21):
    from maleague.components.episode_batch import EpisodeBatch
    B, T1 = arrs["entities"].shape[:2]
    info = {"n_agents": NA, "n_actions": A, "n_entities": NE, "entity_shape": ED, "episode_limit": T1 - 1}
    scheme, groups, pre = entity_scheme_for(info, torch)
    eb = EpisodeBatch(scheme, groups, B, T1, preprocess=pre, device=device)
    for k, v in arrs.items():
        eb.data.transition_data[k].copy_(torch.as_tensor(np.asarray(v)))
    return eb


def _learner(eb, agent_p, mixer_p, args):
    from maleague.controllers import EntityMAC
    from maleague.learners import REFILLearner
    mac = EntityMAC(eb.scheme, eb.groups, args)
    mac.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in agent_p.items()})
    log = _Log()
    L = REFILLearner(mac, eb.scheme, log, args, name="home")
    if mixer_p is not None:
        msd = {k: torch.as_tensor(np.asarray(v)) for k, v in mixer_p.items()}
        L.mixer.load_state_dict(msd)
        L.target_mixer.load_state_dict(msd)
    L.target_mac.load_state(mac)
    L.build_optimizer()
    return L, log


def _pre(d, prefix):
    return {k[len(prefix):]: d[k] for k in d.files if k.startswith(prefix)}


@pytest.mark.parametrize("inst", ["static", "generic"])
def test_refil_learner_two_calls_match_golden(device, golden, inst, monkeypatch):
    """The refil_8 shape runs the static instantiations of the per-item kernels; MLG_REFIL_GENERIC=1 the generic
    ones: both against the reference's two train calls."""
    if inst == "generic":
        monkeypatch.setenv("MLG_REFIL_GENERIC", "1")
    d = golden("refil_learner.npz")
    a = refil_args(device="cuda")
    eb = _batch_from(_pre(d, "b."), device)
    L, log = _learner(eb, _pre(d, "p0.agent."), _pre(d, "p0.mixer."), a)
    for call in range(2):
        L.train(eb, 0, episode_num=call, groupA=torch.from_numpy(d[f"c{call}.groupA"]))
        st = L.last_stats
        for k, v in st.items():
            np.testing.assert_allclose(v, float(d[f"c{call}.stat.{k}"]), rtol=2e-4, atol=1e-6, err_msg=f"call {call} {k}")
        for k, v in L.mac.agent.named_parameters():
            np.testing.assert_allclose(v.detach().cpu().numpy(), d[f"c{call}.agent.{k}"], atol=2e-5, rtol=0,
                                       err_msg=f"call {call} agent {k}")
        for k, v in L.mixer.named_parameters():
            np.testing.assert_allclose(v.detach().cpu().numpy(), d[f"c{call}.mixer.{k}"], atol=2e-5, rtol=0,
                                       err_msg=f"call {call} mixer {k}")
    # the reference REFIL learner logs unprefixed keys (refil_learner.py:185-195), im_loss for imagine agents
    assert set(log.stats) == {"loss", "im_loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"}
    # Agent.trained_steps += mask.sum() per call (refil_learner.py:176), counted by the optimizer launch
    assert L.mac.agent.trained_steps == 2 * int(round(float(L._stats[6].item())))


def test_refil_device_group_draw(device):
    """The imagine group draw on the device (mlg_refil_draw_groups, entity_rnn_agent.py:95-97: p_b ~ U(0,1) per
    episode, entities in group A with probability p_b): deterministic per (seed, draw), fresh per draw, and
    distributed like the reference's draw (overall rate 1/2, per-episode rates spread like U(0,1))."""
    from maleague import _native
    B, NE = 4096, 16
    out = [torch.empty(B, NE, dtype=torch.uint8, device=device) for _ in range(3)]
    for o, draw in zip(out, (7, 7, 8)):
        _native.call("mlg_refil_draw_groups", B, NE, 1234, draw, o.data_ptr(), _native.stream_ptr())
    g = [o.cpu().numpy() for o in out]
    assert np.array_equal(g[0], g[1]) and not np.array_equal(g[0], g[2])
    assert set(np.unique(g[0])) <= {0, 1}
    rate = g[0].mean(axis=1)
    assert abs(rate.mean() - 0.5) < 0.02
    # per-episode rate ~ p_b: variance = Var(p) + E[p(1-p)] / NE = 1/12 + 1/(6 NE)
    assert abs(rate.var() - (1 / 12 + 1 / (6 * NE))) < 0.01
    assert (rate == 0).mean() > 0.01 and (rate == 1).mean() > 0.01


@pytest.mark.parametrize("softmax,double_q", [(False, True), (True, False)])
def test_refil_learner_matches_oracle_on_hip_rollouts(device, softmax, double_q):
    """Episodes from the HIP REFIL rollout (variable 3..8 agents, eps 0.3), random group draws, 2 train calls."""
    from test_gpu_refil import _rollout
    spec, ag, a0, nb, summ, _ = _rollout(device, B=8, T=30, seed=11, eps=0.3, test_mode=False)
    T = int(summ["len"].max()) + 1
    arrs = {k: v[:, :T] for k, v in nb.items() if k != "filled"} | {"filled": nb["filled"][:, :T]}
    a = refil_args(device="cuda", softmax_mixing_weights=softmax, double_q=double_q)
    eb = _batch_from(arrs, device)
    torch.manual_seed(4)
    from maleague.modules.mixers import FlexQMixer
    mixer_p = {k: v.detach().cpu().numpy() for k, v in FlexQMixer(refil_args(device="cpu")).state_dict().items()}
    agent_p = {k: v.detach().cpu().numpy() for k, v in ag.state_dict().items()}
    L, _ = _learner(eb, agent_p, mixer_p, a)
    ref = RR.REFILLearnerRef(agent_p, mixer_p, refil_args(device="cpu", softmax_mixing_weights=softmax,
                                                          double_q=double_q))
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in arrs.items()}
    g = torch.Generator().manual_seed(7)
    for call in range(2):
        groupA = torch.bernoulli(torch.rand(8, 1, 1, generator=g).repeat(1, 1, 16), generator=g).to(torch.uint8)
        want = ref.train(batch, groupA, episode_num=call)
        L.train(eb, 0, episode_num=call, groupA=groupA.to(device))
        got = L.last_stats
        for k in want:
            np.testing.assert_allclose(got[k], want[k], rtol=2e-4, atol=1e-5, err_msg=f"call {call} {k}")
        for k, v in L.mac.agent.named_parameters():
            np.testing.assert_allclose(v.detach().cpu().numpy(), ref.agent[k].detach().numpy(), atol=2e-5, rtol=0,
                                       err_msg=f"call {call} agent {k}")
        for k, v in L.mixer.named_parameters():
            np.testing.assert_allclose(v.detach().cpu().numpy(), ref.mixer[k].detach().numpy(), atol=2e-5, rtol=0,
                                       err_msg=f"call {call} mixer {k}")


def test_refil_learner_padded_steps_are_inert(device, golden):
    """The learner stops at max_t_filled on the device: the golden batch padded with 9 empty timesteps (the
    in-place sampled view's full buffer length) trains exactly like the unpadded one (reference truncation)."""
    d = golden("refil_learner.npz")
    a = refil_args(device="cuda")
    arrs = _pre(d, "b.")
    pad = {k: np.concatenate([v, np.zeros((v.shape[0], 9) + v.shape[2:], v.dtype)], axis=1) for k, v in arrs.items()}
    L1, _ = _learner(_batch_from(arrs, device), _pre(d, "p0.agent."), _pre(d, "p0.mixer."), a)
    L2, _ = _learner(_batch_from(pad, device), _pre(d, "p0.agent."), _pre(d, "p0.mixer."), a)
    for call in range(2):
        g = torch.from_numpy(d[f"c{call}.groupA"])
        L1.train(_batch_from(arrs, device), 0, episode_num=call, groupA=g)
        L2.train(_batch_from(pad, device), 0, episode_num=call, groupA=g)
        s1, s2 = L1.last_stats, L2.last_stats
        for k in s1:
            np.testing.assert_allclose(s2[k], s1[k], rtol=1e-5, atol=1e-7, err_msg=k)
        np.testing.assert_allclose(L2._flat.flat.cpu().numpy(), L1._flat.flat.cpu().numpy(), atol=1e-6, rtol=0)


def test_refil_learner_matches_oracle_config5_batch(device):
    """the config-5 learner shape -- 32 episodes (drawn from a 64-env rollout of the HIP REFIL kernel
    at episode_limit 100, eps 0.05, 3..8 agents per env) truncated at max_t_filled, one train call vs the oracle."""
    from test_gpu_refil import _rollout
    spec, ag, a0, nb, summ, _ = _rollout(device, B=64, T=100, seed=21, eps=0.05, test_mode=False)
    rng = np.random.RandomState(3)
    ids = np.sort(rng.choice(64, 32, replace=False))
    T = int(summ["len"][ids].max()) + 1
    arrs = {k: np.ascontiguousarray(v[ids, :T]) for k, v in nb.items()}
    a = refil_args(device="cuda")
    eb = _batch_from(arrs, device)
    torch.manual_seed(6)
    from maleague.modules.mixers import FlexQMixer
    mixer_p = {k: v.detach().cpu().numpy() for k, v in FlexQMixer(refil_args(device="cpu")).state_dict().items()}
    agent_p = {k: v.detach().cpu().numpy() for k, v in ag.state_dict().items()}
    L, _ = _learner(eb, agent_p, mixer_p, a)
    ref = RR.REFILLearnerRef(agent_p, mixer_p, refil_args(device="cpu"))
    batch = {k: torch.from_numpy(v) for k, v in arrs.items()}
    g = torch.Generator().manual_seed(9)
    groupA = torch.bernoulli(torch.rand(32, 1, 1, generator=g).repeat(1, 1, 16), generator=g).to(torch.uint8)
    want = ref.train(batch, groupA, episode_num=0)
    L.train(eb, 0, episode_num=0, groupA=groupA.to(device))
    got = L.last_stats
    for k in want:
        np.testing.assert_allclose(got[k], want[k], rtol=2e-4, atol=1e-5, err_msg=k)
    for k, v in L.mac.agent.named_parameters():
        np.testing.assert_allclose(v.detach().cpu().numpy(), ref.agent[k].detach().numpy(), atol=2e-5, rtol=0,
                                   err_msg=f"agent {k}")
    for k, v in L.mixer.named_parameters():
        np.testing.assert_allclose(v.detach().cpu().numpy(), ref.mixer[k].detach().numpy(), atol=2e-5, rtol=0,
                                   err_msg=f"mixer {k}")


def test_refil_learner_sampled_view_matches_copy(device):
    """The bench's path: 32 episodes sampled as an in-place view of a device replay buffer (slot map handed to the
    kernels as a kernel argument, MlgRefilLearnerBufs.host_rows) train exactly like the gathered copy of the same
    episodes (no slot map)."""
    from maleague.components.replay_buffer import ReplayBuffer
    from test_gpu_refil import _rollout
    from helpers import entity_scheme_for
    spec, ag, a0, nb, summ, _ = _rollout(device, B=64, T=100, seed=23, eps=0.05, test_mode=False)
    arrs = {k: np.ascontiguousarray(v) for k, v in nb.items()}
    eb = _batch_from(arrs, device)
    B, T1 = arrs["entities"].shape[:2]
    info = {"n_agents": 8, "n_actions": 21, "n_entities": 16, "entity_shape": 8, "episode_limit": T1 - 1}
    scheme, groups, pre = entity_scheme_for(info, torch)
    buf = ReplayBuffer(scheme, groups, 80, T1, preprocess=pre, device=device)
    buf.insert_episode_batch(eb)
    np.random.seed(1)
    view = buf.sample(32, view=True)
    assert view.host_rows is not None and view.host_rows.dtype == np.int32
    copy_ = buf[view.ep_ids]
    a = refil_args(device="cuda")
    torch.manual_seed(8)
    from maleague.modules.mixers import FlexQMixer
    mixer_p = {k: v.detach().cpu().numpy() for k, v in FlexQMixer(refil_args(device="cpu")).state_dict().items()}
    agent_p = {k: v.detach().cpu().numpy() for k, v in ag.state_dict().items()}
    L1, _ = _learner(eb, agent_p, mixer_p, a)
    L2, _ = _learner(eb, agent_p, mixer_p, a)
    g = torch.Generator().manual_seed(12)
    for call in range(2):
        groupA = torch.bernoulli(torch.rand(32, 1, 1, generator=g).repeat(1, 1, 16), generator=g).to(torch.uint8)
        L1.train(view, 0, episode_num=call, groupA=groupA.to(device))
        L2.train(copy_, 0, episode_num=call, groupA=groupA.to(device))
        s1, s2 = L1.last_stats, L2.last_stats
        for k in s1:
            assert s1[k] == s2[k], (call, k, s1[k], s2[k])
        assert torch.equal(L1._flat.flat, L2._flat.flat), call
    assert view._rows is None  # the slot map never went to the device


def _synthetic_entity_batch(B, T1, NA, NE, ED, A, lens, seed):
    """A random entity-scheme batch of any shape (the env variant only produces NA = 8): episode b holds lens[b]
    transitions (filled t <= lens[b], terminated at lens[b] - 1 for even b), a random number of active entities
    (the rest padded: entity_mask 1, zero features), random observability, availability (>= 1 per agent row) and
    actions among the available ones. Keys as EpisodeBatch.transition_data."""
    rng = np.random.RandomState(seed)
    ent = (0.5 * rng.randn(B, T1, NE, ED)).astype(np.float32)
    emask = np.zeros((B, T1, NE), np.uint8)
    omask = (rng.rand(B, T1, NE, NE) < 0.3).astype(np.uint8)
    avail = (rng.rand(B, T1, NA, A) < 0.5).astype(np.int32)
    avail[..., 0] = np.maximum(avail[..., 0], (avail.sum(-1) == 0).astype(np.int32))
    acts = np.zeros((B, T1, NA, 1), np.int64)
    filled = np.zeros((B, T1, 1), np.int64)
    term = np.zeros((B, T1, 1), np.uint8)
    rew = rng.randn(B, T1, 1).astype(np.float32)
    for b in range(B):
        k = rng.randint(max(1, NA - 3), NA + 1)  # active agents
        kn = rng.randint(k, NE + 1)               # active entities
        emask[b, :, kn:] = 1
        emask[b, :, k:NA] = 1
        L = int(lens[b])
        filled[b, :L + 1] = 1
        if b % 2 == 0:
            term[b, L - 1] = 1
        for t in range(T1):
            dead = rng.rand(NE) < 0.1
            emask[b, t, dead] = 1
            for n in range(NA):
                ok = np.nonzero(avail[b, t, n])[0]
                acts[b, t, n, 0] = ok[rng.randint(len(ok))]
        emask[b, L + 1:] = 0
    ent[emask.astype(bool)] = 0.0
    omask = np.maximum(omask, emask[:, :, None, :])
    omask = np.maximum(omask, emask[:, :, :, None])
    for x in (ent, rew, avail, acts):
        for b in range(B):
            x[b, int(lens[b]) + 1:] = 0
    omask[filled[..., 0] == 0] = 0
    emask[filled[..., 0] == 0] = 0
    onehot = np.zeros((B, T1, NA, A), np.float32)
    np.put_along_axis(onehot, acts, 1.0, axis=-1)
    onehot[filled[..., 0] == 0] = 0
    return {"entities": ent, "obs_mask": omask, "entity_mask": emask, "actions": acts, "avail_actions": avail,
            "reward": rew, "terminated": term, "actions_onehot": onehot, "filled": filled}


@pytest.mark.parametrize("NA,NE", [(5, 12), (3, 7)])
def test_refil_learner_na_not_multiple_of_8_matches_oracle(device, NA, NE):
    """the learner's NA % 8 != 0 branch (generic instantiations; no t-major skipping, conditional zeroing
    of d2 / dfc2 / dout) against the oracle: two train calls on a random batch of NA agents among NE entities."""
    A = 5 + NE
    B, T1 = 8, 25
    lens = np.random.RandomState(NA).randint(4, T1 - 1, size=B)
    arrs = _synthetic_entity_batch(B, T1, NA, NE, 8, A, lens, seed=NA * 10 + NE)
    T = int(lens.max()) + 1
    arrs = {k: np.ascontiguousarray(v[:, :T]) for k, v in arrs.items()}
    a_dev = refil_args(device="cuda", n_agents=NA, n_entities=NE, n_actions=A)
    a_cpu = refil_args(device="cpu", n_agents=NA, n_entities=NE, n_actions=A)
    eb = _batch_from(arrs, device, NE=NE, NA=NA, A=A)
    torch.manual_seed(NA)
    from maleague.modules.agents import REGISTRY as agent_REGISTRY
    from maleague.modules.mixers import FlexQMixer
    mixer_p = {k: v.detach().cpu().numpy() for k, v in FlexQMixer(a_cpu).state_dict().items()}
    ag = agent_REGISTRY["imagine_entity_attend_rnn"](8 + A, a_cpu)
    agent_p = {k: v.detach().cpu().numpy() for k, v in ag.state_dict().items()}
    L, _ = _learner(eb, agent_p, mixer_p, a_dev)
    ref = RR.REFILLearnerRef(agent_p, mixer_p, a_cpu)
    batch = {k: torch.from_numpy(v) for k, v in arrs.items()}
    g = torch.Generator().manual_seed(9)
    for call in range(2):
        groupA = torch.bernoulli(torch.rand(B, 1, 1, generator=g).repeat(1, 1, NE), generator=g).to(torch.uint8)
        want = ref.train(batch, groupA, episode_num=call)
        L.train(eb, 0, episode_num=call, groupA=groupA.to(device))
        got = L.last_stats
        for k in want:
            np.testing.assert_allclose(got[k], want[k], rtol=2e-4, atol=1e-5, err_msg=f"NA={NA} call {call} {k}")
        for k, v in L.mac.agent.named_parameters():
            np.testing.assert_allclose(v.detach().cpu().numpy(), ref.agent[k].detach().numpy(), atol=2e-5, rtol=0,
                                       err_msg=f"NA={NA} call {call} agent {k}")
        for k, v in L.mixer.named_parameters():
            np.testing.assert_allclose(v.detach().cpu().numpy(), ref.mixer[k].detach().numpy(), atol=2e-5, rtol=0,
                                       err_msg=f"NA={NA} call {call} mixer {k}")


@pytest.mark.parametrize("NA,NE", [(8, 16), (5, 12)])
def test_refil_learner_no_stale_rows_across_calls(device, NA, NE, monkeypatch):
    """rows the backward kernels skip (items past an episode's live steps) must not carry data from an
    earlier call. One learner trains on a batch of LONG episodes, then on one of SHORT episodes (same buffer length,
    so the same workspace layout); a fresh learner holding the first learner's parameters, RMSprop state and targets
    trains on the short batch alone. Both must end bit-identical (parameters, gradients, stats). Run for the
    side-stream and the one-stream form; those two must agree bit for bit as well."""
    A = 5 + NE
    B, T1 = 8, 41
    long_b = _synthetic_entity_batch(B, T1, NA, NE, 8, A, np.full(B, T1 - 2), seed=1)
    short_b = _synthetic_entity_batch(B, T1, NA, NE, 8, A, np.random.RandomState(2).randint(3, 9, size=B), seed=2)
    a_dev = refil_args(device="cuda", n_agents=NA, n_entities=NE, n_actions=A)
    a_cpu = refil_args(device="cpu", n_agents=NA, n_entities=NE, n_actions=A)
    torch.manual_seed(3)
    from maleague.modules.agents import REGISTRY as agent_REGISTRY
    from maleague.modules.mixers import FlexQMixer
    mixer_p = {k: v.detach().cpu().numpy() for k, v in FlexQMixer(a_cpu).state_dict().items()}
    agent_p = {k: v.detach().cpu().numpy() for k, v in
               agent_REGISTRY["imagine_entity_attend_rnn"](8 + A, a_cpu).state_dict().items()}
    g = torch.Generator().manual_seed(5)
    gA = [torch.bernoulli(torch.rand(B, 1, 1, generator=g).repeat(1, 1, NE), generator=g).to(torch.uint8).to(device)
          for _ in range(2)]
    results = {}
    for mode in ("side", "one"):
        if mode == "one":
            monkeypatch.setenv("MLG_REFIL_ONE_STREAM", "1")
        else:
            monkeypatch.delenv("MLG_REFIL_ONE_STREAM", raising=False)
        e_long = _batch_from(long_b, device, NE=NE, NA=NA, A=A)
        e_short = _batch_from(short_b, device, NE=NE, NA=NA, A=A)
        L1, _ = _learner(e_long, agent_p, mixer_p, a_dev)
        L1.train(e_long, 0, episode_num=0, groupA=gA[0])
        torch.cuda.synchronize()
        L2, _ = _learner(e_short, agent_p, mixer_p, a_dev)
        with torch.no_grad():
            L2._flat.flat.copy_(L1._flat.flat)
            L2._sq.copy_(L1._sq)
            L2._tflat.flat.copy_(L1._tflat.flat)
        L1.train(e_short, 0, episode_num=1, groupA=gA[1])
        L2.train(e_short, 0, episode_num=1, groupA=gA[1])
        torch.cuda.synchronize()
        assert torch.equal(L1._flat.flat, L2._flat.flat), mode
        assert torch.equal(L1._grads, L2._grads), mode
        assert L1.last_stats == L2.last_stats, mode
        results[mode] = (L1._flat.flat.clone(), L1._grads.clone(), L1.last_stats)
    assert torch.equal(results["side"][0], results["one"][0]) and torch.equal(results["side"][1], results["one"][1])
    assert results["side"][2] == results["one"][2]
