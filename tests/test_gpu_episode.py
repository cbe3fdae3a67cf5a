"""BASELINE config 1 -- vanilla QMIX on ma-env 3v3 with runner "episode" (EpisodeStepper, batch_size_run = 1) through
MultiAgentExperiment: the reference's default loop shape (src/steppers/episode_stepper.py:86-171,
src/runs/train/ma_experiment.py:140-241; qmix.yaml / default.yaml: runner "episode"). The PyTorch-CPU flavour of
config 1 has no product path here (every product op is a HIP kernel): it is served by the oracle
baseline (oracle/cpu_baseline.py), and this test runs the same loop on the GPU against that oracle.

Checked: every episode stored in the replay buffer replays bit-exactly through the C env restatement (teacher forced:
obs, state, avail, reward, terminated, filled), t_env = the sum of the episode lengths, one train per run once the
buffer can sample, and the first train call's stats against the PyTorch-CPU QLearner restatement.
"""
import copy

import numpy as np
import pytest
import torch

import learner_ref as LR
from helpers import ref_envs_for

pytestmark = pytest.mark.gpu


def test_config1_episode_runner_through_experiment(device):
    from maleague.custom_logging import MainLogger
    from maleague.runs import MultiAgentExperiment
    from maleague.steppers import EpisodeStepper
    from maleague.utils.config import build_config, to_args
    cfg = build_config("qmix", "ma", overrides=["runner=episode", "batch_size_run=1", "buffer_cpu_only=False",
                                                "buffer_size=64", "batch_size=4", "env_args.match_build_plan=small",
                                                "env_args.episode_limit=40", "t_max=1000000", "test_nepisode=3",
                                                "test_interval=100000000", "seed=3"])
    args = to_args(cfg)
    np.random.seed(0)
    exp = MultiAgentExperiment(args, MainLogger())
    st = exp.stepper
    assert isinstance(st, EpisodeStepper) and st.batch_size == 1
    assert exp.args.n_agents == 3  # 3v3 small.json: the policy team
    learner = exp.home_learner
    captured = {}
    orig_train = learner.train

    def spy(batch, t_env, episode_num):  # the first train call: parameters and the sampled batch before the update
        if not captured:
            captured["agent"] = {k: v.detach().cpu().clone() for k, v in exp.home_mac.agent.state_dict().items()}
            captured["mixer"] = {k: v.detach().cpu().clone() for k, v in learner.mixer.state_dict().items()}
            T = int(batch.max_t_filled())
            captured["batch"] = {k: v[:, :T].detach().cpu().clone() for k, v in batch.data.transition_data.items()}
            captured["t_env"] = int(t_env() if callable(t_env) else t_env)
            captured["episode"] = episode_num
        out = orig_train(batch, t_env, episode_num)
        if "stats" not in captured:
            captured["stats"] = {k: float(learner.last_stats[k]) for k in
                                 ("loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean")}
        return out

    learner.train = spy
    n_it = 10
    exp.start(max_iterations=n_it)
    torch.cuda.synchronize()
    buf = exp.home_buffer
    assert buf.episodes_in_buffer == n_it
    nb = {k: v[:n_it].detach().cpu().numpy() for k, v in buf.data.transition_data.items()}
    ref = ref_envs_for(st.spec, 1, seed=st.spec.seed)[0]
    # the reference tests right after the first training run (last_test_T starts at -test_interval - 1,
    # ma_experiment.py:179-186): test_nepisode // batch_size_run test-mode runs consume env episodes 1..3
    n_test = int(st.envs.episode[0].item()) - n_it
    assert n_test == 3
    total = 0
    for e in range(n_it):  # train episode e of env 0: oracle episode e (e = 0) or e + n_test
        ref.reset()
        if e == 1:
            for _ in range(n_test):
                ref.reset()
        L = int(nb["filled"][e, :, 0].sum()) - 1
        assert 1 <= L <= 40
        np.testing.assert_array_equal(nb["obs"][e, 0], ref.obs())
        np.testing.assert_array_equal(nb["state"][e, 0], ref.state())
        for t in range(L):
            np.testing.assert_array_equal(nb["avail_actions"][e, t], ref.avail())
            rew, done, _ = ref.step(nb["actions"][e, t, :, 0])
            assert nb["reward"][e, t, 0] == np.float32(rew[0]), (e, t)
            assert bool(nb["terminated"][e, t, 0]) == bool(done) == (t == L - 1), (e, t)
            np.testing.assert_array_equal(nb["obs"][e, t + 1], ref.obs(), err_msg=f"obs e={e} t={t}")
            np.testing.assert_array_equal(nb["state"][e, t + 1], ref.state())
        assert nb["filled"][e, L + 1:].sum() == 0
        total += L
    assert st.t_env == total
    # one train per run once the buffer holds batch_size episodes: the first call vs the oracle
    assert captured and captured["episode"] == 3  # iterations 0..3: the 4th run makes the buffer sample
    oracle = LR.QLearnerRef(captured["agent"], captured["mixer"], copy.copy(exp.args))
    want = oracle.train(captured["batch"], captured["t_env"], captured["episode"])
    for k, v in captured["stats"].items():
        assert abs(v - want[k]) <= 2e-4 * abs(want[k]) + 1e-6, (k, v, want[k])
