"""QLearner.train / REFILLearner.train (MODE=refil) microbenchmark on the bench's shapes: 5v5 medium_1h_4t (refil:
refil_8, 3-8 agents) rollouts (ENVS envs, episode_limit 100) fill a device replay ring, then REPS train() calls on
batch_size 32 samples read in place (the bench's path).
Prints mean ms per train() (HIP events on the learner's stream) and the loss of the last call, so variant libraries
(MLG_LIB=...) can be A/B-compared; run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ma-league_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import torch

from maleague.custom_logging import MainLogger
from maleague.runs import MultiAgentExperiment
from maleague.utils.config import build_config, to_args

ENVS = int(os.environ.get("ENVS", "512"))
REPS = int(os.environ.get("REPS", "50"))
overrides = [f"batch_size_run={ENVS}", "runner=parallel", "buffer_cpu_only=False",
             "env_args.match_build_plan=medium_1h_4t", "env_args.episode_limit=100", "seed=0",
             "learner_log_interval=1000000000", "log_interval=1000000000", "runner_log_interval=1000000000",
             "test_interval=1000000000000", "t_max=1000000000000", "show_exp_parameters=False"]
MODE = os.environ.get("MODE", "qmix")
if MODE == "refil":
    overrides = [o.replace("medium_1h_4t", "refil_8") for o in overrides]
    cfg = build_config("refil", "ma_entity", overrides=overrides, device_index=0)
else:
    cfg = build_config("qmix", "ma", overrides=overrides, device_index=0)
np.random.seed(0)
torch.manual_seed(0)
args = to_args(cfg)
exp = MultiAgentExperiment(args, MainLogger(log_interval=10 ** 12))
exp._init_stepper()
exp.stepper.t_env = 10 ** 6
for i in range(2):  # fill the ring (and warm the learner)
    exp._train_episode(i * ENVS)
torch.cuda.synchronize()
buf, lrn = exp.home_buffer, exp.home_learner
samples = [buf.sample(args.batch_size, view=True) for _ in range(REPS)]
lrn.train(samples[0], 10 ** 6, 0)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(REPS)]
for r in range(REPS):
    ev[r][0].record()
    lrn.train(samples[r], 10 ** 6, 0)
    ev[r][1].record()
torch.cuda.synchronize()
ms = [a.elapsed_time(b) for a, b in ev]
print(json.dumps({"train_ms": sum(ms) / len(ms), "min_ms": min(ms), "loss": lrn.last_stats["loss"],
                  "grad_norm": lrn.last_stats["grad_norm"], "T": samples[0].max_seq_length,
                  "t_filled_mean": float(np.mean([int(s_.max_t_filled()) for s_ in samples[:10]]))}))
