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
buf = torch.zeros(grid * 8 * 32 + grid * 128, dtype=torch.int64, device="cuda")  # phase slots + step trace
_native.call("mlg_debug_set_stamps", _native.ptr(buf))
for it in range(3):
    buf.zero_()
    exp._train_episode(it * B)
torch.cuda.synchronize()
allb = buf.cpu().numpy()
a = allb[:grid * 256].reshape(grid, 8, 32).astype(np.float64)
tr = allb[grid * 256:].reshape(grid, 128)
valid = a[:, :, 31] == 1
if os.environ.get("MLG_ROLLOUT_KERNEL", "v4") == "v1":
    names = ["agent", "barrier_after_agent", "-", "-"]
    names += ["E1_exec_actions", "E2_resolve(+bar)", "E3_reduce(+bar)", "obs(+bar)", "state", "avail",
              "zero+list+barrier"]
elif os.environ.get("MLG_ROLLOUT_KERNEL", "v4") == "v7":
    names = ["A_fc1", "B_gru", "C_fc2_select", "barrier_after_C", "E1_exec(+E2)", "barrier_A",
             "E3_reduce", "pair_pass", "status/tail-zero", "obs", "barrier_end", "avail", "state", "barrier_B", "rowmap"]
else:
    names = ["A_fc1", "B_gru(+barrier A)", "C_fc2_select(+barrier B)", "barrier_after_C", "E1_exec", "E2_resolve",
             "E3_reduce", "pair_pass", "status/tail-zero", "obs", "barrier_end", "avail", "state"]
if os.environ.get("MLG_ROLLOUT_KERNEL", "v4") == "v4":
    for role, ws in (("agent waves 0-3", slice(0, 4)), ("env waves 4-7", slice(4, 8))):
        sub = a[:, ws, :]
        vv = sub[:, :, 31] == 1
        tt = sub[:, :, 30][vv].mean()
        print(f"-- {role}: mean total {tt:.0f}")
        for k in range(14):
            m = sub[:, :, k][vv].mean()
            if m > 0:
                print(f"   slot {k:2d} mean={m:12.0f} share={m / tt * 100:6.1f}%")
tot = a[:, :, 30][valid].mean()
print(f"rollout waves={valid.sum()} mean total cycles/wave={tot:.0f} (~{tot / 2.1e3:.1f} us at 2.1GHz)")
for k, n in enumerate(names):
    v = a[:, :, k][valid]
    print(f"{n:22s} mean={v.mean():12.0f} share={v.mean() / tot * 100:6.1f}%  max={v.max():.0f}")
tw = a[:, 0, 30][valid[:, 0]]
print("per-WG total cycles: min %.0f p10 %.0f p50 %.0f p90 %.0f max %.0f" % tuple(np.percentile(tw, [0, 10, 50, 90, 100])))
lens = st.last_run["ep_len"].numpy()
wmax = np.array([lens[i:i + 16].max() + 1 for i in range(0, B, 16)])
print("per-WG iterations: min %d p10 %d p50 %d p90 %d max %d" % tuple(np.percentile(wmax, [0, 10, 50, 90, 100]).astype(int)))
print("active env-steps per WG (sum len): p50 %d max %d" % (np.median([lens[i:i+16].sum() for i in range(0, B, 16)]),
      max(lens[i:i+16].sum() for i in range(0, B, 16))))
print("episode len mean", lens.mean(), "max", lens.max(), "iterations per WG (mean of max)",
      np.mean([lens[i:i + 16].max() + 1 for i in range(0, B, 16)]))

# step trace: entry t = (cycles of step t-1) << 8 | running envs at step t
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
mr = int(os.environ.get("MINRUN", "0"))
if mr:  # libmaleague built with -DMLG_STAMPS_MINRUN=mr: phase slots per counted step
    nfull = (nrun >= mr).sum(1).mean()
    print(f"steps with >= {mr} running envs per WG: {nfull:.1f}; per-step phase cycles (mean over waves):")
    for k, n in enumerate(names):
        print(f"  {n:22s} {a[:, :, k][valid].mean() / nfull:8.0f}")
tot_wg = cyc[:, 1:].sum(1)
slow = int(np.argmax(tot_wg))
print("slowest WG", slow, "total", tot_wg[slow], "mean WG", tot_wg.mean())
prof = [(int(nrun[slow, t]), int(cyc[slow, t + 1])) for t in range(127) if nrun[slow, t] > 0]
print("slowest WG steps (nrun, cycles):", prof)
if int(os.environ.get("TIMELINE", "0")):
    # -DMLG_STAMPS_TIMELINE build: slot k = cycles from the start of the WG's first one-env step to mark k
    order = [(0, "fc1"), (5, "barrier_A"), (1, "gru"), (13, "barrier_B"), (2, "fc2"), (3, "barrier_C"),
             (4, "E1E2"), (6, "E3"), (7, "pair"), (9, "obs"), (11, "avail"), (12, "state"), (8, "tail"), (10, "end")]
    envw, oth, w0 = [], [], []
    for g in range(grid):
        for w in range(8):
            if a[g, w, 31] != 1 or a[g, w, 10] == 0:
                continue
            (envw if a[g, w, 7] > 0 else oth).append(a[g, w, :15])
            if w == 0 and a[g, w, 7] == 0:  # wave 0 holds the one tile's fc2 in a one-env step (wave < tiles)
                w0.append(a[g, w, :15])
    for nm, rows in (("env wave", envw), ("other waves", oth), ("wave 0 (fc2 tile, no env)", w0)):
        if not rows:
            continue
        r = np.array(rows)
        print(f"timeline of the first one-env step, {nm} (n={len(r)}): " +
              ", ".join(f"{n}@{r[:, k].mean():.0f}" for k, n in order))
