"""Checkpoint interoperability with the reference.

Fixtures (tests/golden/make_golden.py::checkpoint_fixture): `ckpt_qmix/100/home_qlearner_{agent,mixer,opt}.th`
were written by the reference's QLearner.save_models (src/marl/learners/q_learner.py:133-137,
basic_controller.py:68-69) after one train() call; `checkpoint.npz` holds what a fresh reference learner
did after resuming from them (load_models, q_learner.py:139-147) and training once more.

CPU: our learner loads the reference files (weights_only=True) into its flat parameter / RMSprop buffers,
our own save_models writes files with the reference's names, keys, shapes and optimizer-state structure,
and MultiAgentExperiment finds the latest step directory like run_utils.find_latest_model_path.
GPU: resuming from the reference checkpoint and training once reproduces the reference's resumed call
(stats rtol 1e-4, parameters atol 2e-5 -- the tolerances of test_gpu_learner.py).
"""
import os

import numpy as np
import pytest
import torch

from helpers import qmix_args, scheme_for

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CKPT = os.path.join(GOLD, "ckpt_qmix")


def _load(name):
    return torch.load(os.path.join(CKPT, "100", f"home_qlearner_{name}.th"), map_location="cpu", weights_only=True)


class _Log:
    def __init__(self):
        self.stats = {}

    def log_stat(self, k, v, t):
        self.stats[k] = v

    def info(self, *a):
        pass


def _fresh_learner(device):
    from maleague.components.episode_batch import EpisodeBatch
    from maleague.controllers import BasicMAC
    from maleague.learners import QLearner
    args = qmix_args(device=str(device))
    info = {"state_shape": 60, "obs_shape": 80, "n_actions": 15, "n_agents": 5}
    scheme, groups, preprocess = scheme_for(info, torch)
    proto = EpisodeBatch(scheme, groups, 1, 2, preprocess=preprocess, device=device)
    torch.manual_seed(1234)  # deliberately different from the reference's init: everything must come from the files
    mac = BasicMAC(proto.scheme, groups, args)
    learner = QLearner(mac, proto.scheme, _Log(), args, name="home")
    learner.build_optimizer()
    return learner, args


def test_loads_reference_checkpoint_cpu():
    learner, _ = _fresh_learner(torch.device("cpu"))
    learner.load_models(os.path.join(CKPT, "100"))
    agent, mixer, opt = _load("agent"), _load("mixer"), _load("opt")
    for k, v in learner.mac.agent.state_dict().items():
        assert torch.equal(v, agent[k]), k
    for k, v in learner.target_mac.agent.state_dict().items():  # q_learner.py:142: target MAC loads the same file
        assert torch.equal(v, agent[k]), k
    for k, v in learner.mixer.state_dict().items():
        assert torch.equal(v, mixer[k]), k
    # the loaded RMSprop state lives in the flat square_avg buffer the fused kernel updates
    params = learner.parameters()
    assert len(params) == len(opt["state"])
    for i, p in enumerate(params):
        st = learner.optimiser.state[p]
        assert torch.equal(st["square_avg"], opt["state"][i]["square_avg"]), i
        assert float(st["step"]) == float(opt["state"][i]["step"])
        assert st["square_avg"].data_ptr() >= learner._sq.data_ptr()
    assert torch.equal(learner._flat.flat[:agent["fc1.weight"].numel()], agent["fc1.weight"].reshape(-1))
    assert learner.optimiser.param_groups[0]["lr"] == opt["param_groups"][0]["lr"]


def test_save_matches_reference_format(tmp_path):
    learner, _ = _fresh_learner(torch.device("cpu"))
    learner.load_models(os.path.join(CKPT, "100"))
    learner.save_models(str(tmp_path), learner.name)
    assert sorted(os.listdir(tmp_path)) == sorted(os.listdir(os.path.join(CKPT, "100")))
    for name in ["agent", "mixer"]:
        ours = torch.load(tmp_path / f"home_qlearner_{name}.th", weights_only=True)
        ref = _load(name)
        assert list(ours.keys()) == list(ref.keys())
        for k in ref:
            assert ours[k].dtype == ref[k].dtype and ours[k].shape == ref[k].shape, k
            assert torch.equal(ours[k], ref[k]), k
            assert ours[k].untyped_storage().nbytes() == ref[k].nbytes, k  # no flat-buffer storage in the file
    ours, ref = torch.load(tmp_path / "home_qlearner_opt.th", weights_only=True), _load("opt")
    assert sorted(ours.keys()) == sorted(ref.keys())
    assert ours["param_groups"][0]["params"] == ref["param_groups"][0]["params"]
    for key in ["lr", "alpha", "eps", "weight_decay", "momentum", "centered"]:
        assert ours["param_groups"][0][key] == ref["param_groups"][0][key], key
    assert sorted(ours["state"].keys()) == sorted(ref["state"].keys())
    for i in ref["state"]:
        assert set(ours["state"][i].keys()) == set(ref["state"][i].keys())
        assert torch.equal(ours["state"][i]["square_avg"], ref["state"][i]["square_avg"])
        # a checkpoint must not alias our flat buffer (torch.save of a view stores the whole storage)
        assert ours["state"][i]["square_avg"].untyped_storage().nbytes() == ref["state"][i]["square_avg"].nbytes


def test_experiment_finds_latest_step(tmp_path):
    from maleague.runs.ma_experiment import find_latest_model_path
    for t in [50, 100, 2000]:
        (tmp_path / str(t)).mkdir()
    (tmp_path / "notastep").mkdir()
    assert find_latest_model_path(str(tmp_path)) == (str(tmp_path / "2000"), 2000)
    assert find_latest_model_path(str(tmp_path), 90) == (str(tmp_path / "100"), 100)
    assert find_latest_model_path(CKPT) == (os.path.join(CKPT, "100"), 100)


@pytest.mark.gpu
def test_resume_from_reference_checkpoint_gpu(device, golden):
    """Reference resume (fresh learner + load_models + train) reproduced on the fused HIP learner."""
    import learner_ref as LR
    from maleague.components.episode_batch import EpisodeBatch
    d = golden("checkpoint.npz")
    learner, args = _fresh_learner(device)
    learner.load_models(os.path.join(CKPT, "100"))
    # load_models leaves the target mixer at the fresh learner's init (q_learner.py:139-147); take the reference's
    learner.target_mixer.load_state_dict({k[3:]: torch.from_numpy(np.array(d[k])) for k in d.files
                                          if k.startswith("tm.")})
    b = LR.batch_from_npz(d)
    B, T = b["obs"].shape[:2]
    info = {"state_shape": 60, "obs_shape": 80, "n_actions": 15, "n_agents": 5}
    scheme, groups, preprocess = scheme_for(info, torch)
    eb = EpisodeBatch(scheme, groups, B, T, preprocess=preprocess, device=device)
    for k, v in b.items():
        eb.data.transition_data[k].copy_(v)
    learner.train(eb, 200, 32)
    for k in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
        np.testing.assert_allclose(learner.last_stats[k], float(d[f"stat.{k}"]), rtol=1e-4, atol=1e-6, err_msg=k)
    for prefix, module in [("p2.agent.", learner.mac.agent), ("p2.target_agent.", learner.target_mac.agent),
                           ("p2.mixer.", learner.mixer)]:
        for k, v in module.state_dict().items():
            np.testing.assert_allclose(v.cpu().numpy(), d[prefix + k], atol=2e-5, rtol=0, err_msg=prefix + k)
