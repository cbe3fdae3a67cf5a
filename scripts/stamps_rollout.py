"""Diagnostic: per-phase cycle shares of the rollout kernel (needs libmaleague_stamps.so, MLG_LIB set)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ma-league_amd"), ROOT]
import numpy as np
import torch

from maleague import _native
from maleague.custom_logging import MainLogger
from maleague.runs import MultiAgentExperiment
from maleague.utils.config import build_config, to_args

B = int(os.environ.get("ENVS", "4096"))
cfg = build_config("qmix", "ma", overrides=[f"batch_size_run={B}", "runner=parallel", "buffer_cpu_only=False",
                                           "env_args.episode_limit=100", "show_exp_parameters=False"])
exp = MultiAgentExperiment(to_args(cfg), MainLogger(log_interval=10 ** 12))
exp._init_stepper()
st = exp.stepper
st.t_env = 10 ** 6
grid = (B + 15) // 16
buf = torch.zeros(grid * 8 * 16, dtype=torch.int64, device="cuda")
_native.call("mlg_debug_set_stamps", _native.ptr(buf))
for it in range(3):
    buf.zero_()
    exp._train_episode(it * B)
torch.cuda.synchronize()
a = buf.view(grid, 8, 16).cpu().numpy().astype(np.float64)
valid = a[:, :, 15] == 1
if os.environ.get("MLG_ROLLOUT_KERNEL", "v2") == "v1":
    names = ["agent", "barrier_after_agent", "-", "-"]
    names += ["E1_exec_actions", "E2_resolve(+bar)", "E3_reduce(+bar)", "obs(+bar)", "state", "avail",
              "zero+list+barrier"]
else:
    names = ["A_fc1", "B_gru(+barrier A)", "C_fc2_select(+barrier B)", "barrier_after_C", "E1_exec", "E2_resolve",
             "E3_reduce", "pairs+obs/state/avail", "status", "-", "barrier_end"]
tot = a[:, :, 14][valid].mean()
print(f"rollout waves={valid.sum()} mean total cycles/wave={tot:.0f} (~{tot / 2.1e3:.1f} us at 2.1GHz)")
for k, n in enumerate(names):
    v = a[:, :, k][valid]
    print(f"{n:22s} mean={v.mean():12.0f} share={v.mean() / tot * 100:6.1f}%  max={v.max():.0f}")
lens = st.last_run["ep_len"].numpy()
print("episode len mean", lens.mean(), "max", lens.max(), "iterations per WG (mean of max)",
      np.mean([lens[i:i + 16].max() + 1 for i in range(0, B, 16)]))
