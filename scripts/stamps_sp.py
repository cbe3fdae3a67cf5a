"""Diagnostic: per-phase cycle shares of the self-play rollout kernel (config 3 shape: 5v5, both teams policy
controlled, 4096 envs, episode_limit 100). Needs libmaleague_stamps.so (MLG_LIB set)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ma-league_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import torch

from maleague import _native
from maleague.components.episode_batch import EpisodeBatch
from maleague.controllers import BasicMAC
from maleague.custom_logging import MainLogger
from maleague.envs.plans import builtin_plan
from maleague.steppers import SelfPlayParallelStepper
from helpers import qmix_args, scheme_for

B = int(os.environ.get("ENVS", "4096"))
RS = int(os.environ.get("SP_RS", "8"))  # envs per workgroup of the kernel under test
args = qmix_args(batch_size_run=B, seed=0,
                 env_args={"match_build_plan": builtin_plan("medium_1h_4t", self_play=True), "grid_size": 20,
                           "stochastic_spawns": True, "episode_limit": 100})
stepper = SelfPlayParallelStepper(args, MainLogger())
info = stepper.get_env_info()
args.n_agents, args.n_actions, args.state_shape = info["n_agents"] // 2, info["n_actions"], info["state_shape"]
scheme, groups, preprocess = scheme_for(dict(info, n_agents=args.n_agents), torch)
proto = EpisodeBatch(scheme, groups, 1, 2, preprocess=preprocess, device="cuda")
torch.manual_seed(0)
home, away = BasicMAC(proto.scheme, groups, args), BasicMAC(proto.scheme, groups, args)
stepper.initialize(scheme, groups, preprocess, home, away)
stepper.t_env = 10 ** 6
grid = (B + RS - 1) // RS
buf = torch.zeros(grid * 8 * 32 + grid * 128, dtype=torch.int64, device="cuda")
_native.call("mlg_debug_set_stamps", _native.ptr(buf))
for it in range(3):
    buf.zero_()
    stepper.run(test_mode=False)
torch.cuda.synchronize()
allb = buf.cpu().numpy()
a = allb[:grid * 256].reshape(grid, 8, 32).astype(np.float64)
tr = allb[grid * 256:].reshape(grid, 128)
valid = a[:, :, 31] == 1
names = os.environ.get("SP_SLOTS", "fc1,barrier_A,gru,barrier_B,fc2_select,barrier_C,E1_E2,E3_pair_obs,tail,barrier_end")
names = names.split(",")
tot = a[:, :, 30][valid].mean()
print(f"waves={valid.sum()} mean total cycles/wave={tot:.0f}")
for role, ws in (("waves 0-3", slice(0, 4)), ("waves 4-7", slice(4, 8))):
    sub = a[:, ws, :]
    vv = sub[:, :, 31] == 1
    tt = sub[:, :, 30][vv].mean()
    print(f"-- {role}: mean total {tt:.0f}")
    for k, n in enumerate(names):
        m = sub[:, :, k][vv].mean()
        print(f"   {n:16s} mean={m:12.0f} share={m / tt * 100:6.1f}%")
lens = stepper.last_run["ep_len"].numpy()
print("episode len mean", lens.mean(), "max", lens.max(), "draw-limit share", (lens == 100).mean())
cyc = (tr >> 8).astype(np.float64)
nrun = (tr & 255).astype(np.int64)
by = {}
for g in range(grid):
    for t in range(127):
        if nrun[g, t] == 0 or cyc[g, t + 1] == 0:
            continue
        by.setdefault(int(nrun[g, t]), []).append(cyc[g, t + 1])
print("step cycles by running envs in the WG (mean, count):")
for k in sorted(by):
    print(f"  nrun={k:2d} mean={np.mean(by[k]):8.0f} n={len(by[k])}")
steps = (nrun > 0).sum(1)
print("steps per WG: min %d p50 %d max %d" % (steps.min(), np.median(steps), steps.max()))
