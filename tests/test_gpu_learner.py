"""GPU parity of the fused QLearner.train pipeline (mlg_qlearner_train) against golden vectors of the
reference QLearner (3 consecutive train() calls incl. a hard target update) and against the CPU oracle
(oracle/learner_ref.py) on rollouts produced by the HIP stepper.

Tolerances (fp32, different summation orders): stats rtol 1e-4; parameters after RMSprop atol 2e-5
(RMSprop's first step moves every weight by ~lr * 10 * sign(g), so sign-level agreement of the
gradients is what these checks exercise); north_star's 1e-4 bound on Q-values is asserted on Q.
"""
import copy

import numpy as np
import pytest
import torch

import learner_ref as LR
from helpers import qmix_args, scheme_for

pytestmark = pytest.mark.gpu


def _golden_batch(d, device):
    from maleague.components.episode_batch import EpisodeBatch
    b = LR.batch_from_npz(d)
    B, T, N, _ = b["obs"].shape
    A = b["avail_actions"].shape[-1]
    info = {"state_shape": b["state"].shape[-1], "obs_shape": b["obs"].shape[-1], "n_actions": A, "n_agents": N}
    scheme, groups, preprocess = scheme_for(info, torch)
    eb = EpisodeBatch(scheme, groups, B, T, preprocess=preprocess, device=device)
    for k, v in b.items():
        eb.data.transition_data[k].copy_(v)
    return eb


class _Log:
    def __init__(self):
        self.stats = {}

    def log_stat(self, k, v, t):
        self.stats[k] = v

    def info(self, *a):
        pass


def _learner(d, device, args, mixer_prefix="p0.mixer."):
    from maleague.controllers import BasicMAC
    from maleague.learners import QLearner
    eb = _golden_batch(d, device)
    mac = BasicMAC(eb.scheme, eb.groups, args)
    mac.load_state_dict({k[len("p0.agent."):]: torch.from_numpy(np.array(d[k])) for k in d.files
                         if k.startswith("p0.agent.")})
    log = _Log()
    learner = QLearner(mac, eb.scheme, log, args, name="home")
    if args.mixer == "qmix":
        msd = {k[len(mixer_prefix):]: torch.from_numpy(np.array(d[k])) for k in d.files if k.startswith(mixer_prefix)}
        learner.mixer.load_state_dict(msd)
        learner.target_mixer.load_state_dict(msd)
    learner.build_optimizer()
    return learner, eb, log


@pytest.mark.parametrize("name,kw", [("qlearner_qmix_dq.npz", {}), ("qlearner_qmix_nodq.npz", {"double_q": False}),
                                     ("qlearner_vdn.npz", {"mixer": "vdn"})])
def test_qlearner_golden(device, golden, name, kw):
    d = golden(name)
    args = qmix_args(**kw)
    learner, eb, log = _learner(d, device, args)
    for i, (t_env, ep) in enumerate(d["calls"]):
        learner.train(eb, int(t_env), int(ep))
        for k in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
            np.testing.assert_allclose(learner.last_stats[k], float(d[f"stat{i}.{k}"]), rtol=1e-4, atol=1e-6,
                                       err_msg=f"{name} call {i} {k}")
        assert log.stats["home_qlearner_loss"] == learner.last_stats["loss"]
    last = len(d["calls"])
    sd = learner.mac.agent.state_dict()
    for k, v in sd.items():
        np.testing.assert_allclose(v.cpu().numpy(), d[f"p{last}.agent.{k}"], atol=2e-5, rtol=0, err_msg=k)
    tsd = learner.target_mac.agent.state_dict()
    for k, v in tsd.items():
        np.testing.assert_allclose(v.cpu().numpy(), d[f"p{last}.target_agent.{k}"], atol=2e-5, rtol=0, err_msg=k)
    if args.mixer == "qmix":
        for k, v in learner.mixer.state_dict().items():
            np.testing.assert_allclose(v.cpu().numpy(), d[f"p{last}.mixer.{k}"], atol=2e-5, rtol=0, err_msg=k)
    assert learner.mac.agent.trained_steps == int(d["trained_steps"])


def test_qlearner_vs_oracle_on_rollout(device):
    """Train on a batch produced by the HIP stepper (5v5, 32 episodes) and compare one step with the oracle."""
    from maleague.components.episode_batch import EpisodeBatch
    from maleague.controllers import BasicMAC
    from maleague.custom_logging import MainLogger
    from maleague.learners import QLearner
    from maleague.steppers import ParallelStepper
    args = qmix_args(batch_size_run=32, seed=11, env_args={"match_build_plan": "medium_1h_2t_2a", "grid_size": 20,
                                                           "stochastic_spawns": True, "episode_limit": 60})
    stepper = ParallelStepper(args, MainLogger())
    info = stepper.get_env_info()
    args.n_agents, args.n_actions, args.state_shape = info["n_agents"], info["n_actions"], info["state_shape"]
    scheme, groups, preprocess = scheme_for(info, torch)
    proto = EpisodeBatch(scheme, groups, 1, 2, preprocess=preprocess, device=device)
    torch.manual_seed(3)
    mac = BasicMAC(proto.scheme, groups, args)
    learner = QLearner(mac, proto.scheme, _Log(), args, name="home")
    agent0 = {k: v.detach().cpu().clone() for k, v in mac.agent.state_dict().items()}
    mixer0 = {k: v.detach().cpu().clone() for k, v in learner.mixer.state_dict().items()}
    learner.build_optimizer()
    stepper.initialize(scheme, groups, preprocess, mac)
    stepper.t_env = 30000
    batch, _ = stepper.run(test_mode=False)
    T = int(batch.max_t_filled())
    sample = batch[:, :T]
    ref = LR.QLearnerRef(agent0, mixer0, copy.copy(args))
    tb = {k: v.detach().cpu().clone() for k, v in sample.data.transition_data.items()}
    exp = ref.train(tb, 30000, 0)
    learner.train(sample, 30000, 0)
    for k in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
        np.testing.assert_allclose(learner.last_stats[k], exp[k], rtol=2e-4, atol=1e-6, err_msg=k)
    for k, v in learner.mac.agent.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), ref.agent_state()[k].numpy(), atol=5e-5, rtol=0, err_msg=k)
    for k, v in learner.mixer.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), ref.mixer_state()[k].numpy(), atol=5e-5, rtol=0, err_msg=k)
    # Q of the trained agent within 1e-4 of the oracle forward with the same (updated) weights
    q_ref, _ = LR.mac_unroll({k: v.detach().cpu() for k, v in learner.mac.agent.state_dict().items()}, tb,
                             args.n_agents, T=T)
    learner.mac.init_hidden(sample.batch_size)
    for t in range(T):
        q = learner.mac.forward(sample, t)
        np.testing.assert_allclose(q.cpu().numpy(), q_ref[:, t].numpy(), atol=1e-4, rtol=0)


def test_qlearner_sampled_view_equals_truncated_copy(device):
    """QLearner.train on a SampledEpisodeBatch (in-place slot-map read of the device replay buffer, full stored
    length) matches train on the reference path's gathered copy truncated to max_t_filled: same loss, stats,
    updated parameters (fp32 summation order only) and trained_steps."""
    from maleague.components.episode_batch import EpisodeBatch
    from maleague.components.replay_buffer import ReplayBuffer
    from maleague.controllers import BasicMAC
    from maleague.custom_logging import MainLogger
    from maleague.learners import QLearner
    from maleague.steppers import ParallelStepper
    args = qmix_args(batch_size_run=48, seed=4, env_args={"match_build_plan": "medium_1h_4t", "grid_size": 20,
                                                          "stochastic_spawns": True, "episode_limit": 50})
    stepper = ParallelStepper(args, MainLogger())
    info = stepper.get_env_info()
    args.n_agents, args.n_actions, args.state_shape = info["n_agents"], info["n_actions"], info["state_shape"]
    scheme, groups, preprocess = scheme_for(info, torch)
    buf = ReplayBuffer(scheme, groups, 100, 64, preprocess=preprocess, device=device)  # longer than episodes
    torch.manual_seed(5)
    learners = []
    for _ in range(2):
        torch.manual_seed(5)
        mac = BasicMAC(buf.scheme, groups, args)
        lrn = QLearner(mac, buf.scheme, _Log(), args, name="home")
        lrn.build_optimizer()
        learners.append(lrn)
    stepper.initialize(scheme, groups, preprocess, learners[0].mac)
    assert not stepper.attach_replay(buf)  # different length: plain inserts
    stepper.t_env = 20000
    for _ in range(3):  # 144 episodes into a 100-slot ring (wraps)
        b, _ = stepper.run(test_mode=False)
        buf.insert_episode_batch(b)
    np.random.seed(0)
    view = buf.sample(32, view=True)
    assert view.max_seq_length == 64 and view.rows.dtype == torch.int32
    copy_ = buf[view.ep_ids]
    T = int(copy_.max_t_filled())
    assert T <= 51
    learners[0].train(view, lambda: 1, 0)
    learners[1].train(copy_[:, :T], 1, 0)
    s0, s1 = learners[0].last_stats, learners[1].last_stats
    for k in s0:
        np.testing.assert_allclose(s0[k], s1[k], rtol=1e-5, atol=1e-7, err_msg=k)
    for (k, v0), v1 in zip(learners[0].mac.agent.state_dict().items(), learners[1].mac.agent.state_dict().values()):
        np.testing.assert_allclose(v0.cpu().numpy(), v1.cpu().numpy(), atol=1e-6, rtol=0, err_msg=k)
    for (k, v0), v1 in zip(learners[0].mixer.state_dict().items(), learners[1].mixer.state_dict().values()):
        np.testing.assert_allclose(v0.cpu().numpy(), v1.cpu().numpy(), atol=1e-6, rtol=0, err_msg=k)
    assert learners[0].mac.agent.trained_steps == learners[1].mac.agent.trained_steps > 0
    # host reads of the view materialise the same episodes
    for k in ("obs", "actions", "filled"):
        assert torch.equal(view[k], copy_[k]), k


def test_qlearner_vs_oracle_full_config2_sample(device):
    """the config-2 shapes -- a 4096-env, episode_limit 100 train-mode rollout written into the HBM
    replay ring, 32 episodes sampled in place (the learner reads the slot map over the buffer's full length), one
    QLearner.train against the oracle on the truncated gathered copy of the same 32 episodes."""
    from maleague.components.episode_batch import EpisodeBatch
    from maleague.components.replay_buffer import ReplayBuffer
    from maleague.controllers import BasicMAC
    from maleague.custom_logging import MainLogger
    from maleague.learners import QLearner
    from maleague.steppers import ParallelStepper
    B = 4096
    args = qmix_args(batch_size_run=B, seed=7, env_args={"match_build_plan": "medium_1h_4t", "grid_size": 20,
                                                         "stochastic_spawns": True, "episode_limit": 100})
    stepper = ParallelStepper(args, MainLogger())
    info = stepper.get_env_info()
    args.n_agents, args.n_actions, args.state_shape = info["n_agents"], info["n_actions"], info["state_shape"]
    scheme, groups, preprocess = scheme_for(info, torch)
    proto = EpisodeBatch(scheme, groups, 1, 2, preprocess=preprocess, device=device)
    torch.manual_seed(5)
    mac = BasicMAC(proto.scheme, groups, args)
    learner = QLearner(mac, proto.scheme, _Log(), args, name="home")
    agent0 = {k: v.detach().cpu().clone() for k, v in mac.agent.state_dict().items()}
    mixer0 = {k: v.detach().cpu().clone() for k, v in learner.mixer.state_dict().items()}
    learner.build_optimizer()
    stepper.initialize(scheme, groups, preprocess, mac)
    ring = ReplayBuffer(scheme, groups, 5000, 101, preprocess=preprocess, device=device)
    assert stepper.attach_replay(ring)
    stepper.t_env = 10 ** 6  # epsilon floor 0.05
    batch, _ = stepper.run(test_mode=False)
    ring.insert_episode_batch(batch)
    np.random.seed(4)
    sample = ring.sample(32, view=True)
    T = int(sample.max_t_filled())
    assert T >= 30
    tb = {k: v[:, :T].detach().cpu().clone() for k, v in sample.data.transition_data.items()}
    ref = LR.QLearnerRef(agent0, mixer0, copy.copy(args))
    want = ref.train(tb, 10 ** 6, 0)
    learner.train(sample, 10 ** 6, 0)
    for k in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
        np.testing.assert_allclose(learner.last_stats[k], want[k], rtol=2e-4, atol=1e-6, err_msg=k)
    for k, v in learner.mac.agent.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), ref.agent_state()[k].numpy(), atol=5e-5, rtol=0, err_msg=k)
    for k, v in learner.mixer.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), ref.mixer_state()[k].numpy(), atol=5e-5, rtol=0, err_msg=k)


def test_qlearner_small_gate_preactivations(device, golden):
    """the fused learner's gates run on v_exp / v_rcp with tanh(x) = 2 sigmoid(2x) - 1, which loses
    relative precision for small |x|. GRU weights and biases scaled by 1e-3 (every gate pre-activation |x| << 1,
    n ~ tanh of tiny values): stats and updated parameters still within the learner bars of the oracle."""
    d = golden("qlearner_qmix_dq.npz")
    args = qmix_args()
    agent0 = {k[len("p0.agent."):]: np.array(d[k]) for k in d.files if k.startswith("p0.agent.")}
    for k in list(agent0):
        if k.startswith("gru."):
            agent0[k] = (agent0[k] * 1e-3).astype(np.float32)
    mixer0 = {k[len("p0.mixer."):]: np.array(d[k]) for k in d.files if k.startswith("p0.mixer.")}
    dd = {("p0.agent." + k): v for k, v in agent0.items()} | {("p0.mixer." + k): v for k, v in mixer0.items()}

    class _D(dict):
        files = property(lambda self: list(self.keys()))

    src = _D({k: d[k] for k in d.files if not k.startswith("p0.")} | dd)
    learner, eb, log = _learner(src, device, args)
    ref = LR.QLearnerRef(agent0, mixer0, copy.copy(args))
    tb = {k: v.detach().cpu().clone() for k, v in eb.data.transition_data.items()}
    want = ref.train(tb, 0, 0)
    learner.train(eb, 0, 0)
    for k in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
        np.testing.assert_allclose(learner.last_stats[k], want[k], rtol=1e-4, atol=1e-7, err_msg=k)
    for k, v in learner.mac.agent.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), ref.agent_state()[k].numpy(), atol=2e-5, rtol=0, err_msg=k)
