"""Diagnostic: per-phase cycle shares of the REFIL rollout kernel (needs libmaleague_stamps.so via MLG_LIB)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ma-league_amd"), os.path.join(ROOT, "tests")]
from helpers import entity_scheme_for, refil_args  # noqa: E402
from maleague import _native  # noqa: E402
from maleague.components.batch_view import mlg_entity_batch  # noqa: E402
from maleague.components.episode_batch import EpisodeBatch  # noqa: E402
from maleague.envs.entity_env import EntityEnvSpec  # noqa: E402
from maleague.envs.teams_env import VecEnvState  # noqa: E402
from maleague.modules.agents import REGISTRY  # noqa: E402

B = int(os.environ.get("B", 4096))
dev = torch.device("cuda:0")
spec = EntityEnvSpec.from_env_args({"match_build_plan": "refil_8", "episode_limit": 100, "seed": 0})
torch.manual_seed(0)
ag = REGISTRY["imagine_entity_attend_rnn"](29, refil_args()).to(dev)
scheme, groups, pre = entity_scheme_for(spec.env_info(), torch)
batch = EpisodeBatch(scheme, groups, B, 101, preprocess=pre, device=dev)
mb, keep = mlg_entity_batch(batch)
mb.full_write = 1
st = VecEnvState(spec, B, dev)
run = torch.zeros(6 * B, dtype=torch.int32, device=dev)
ri = _native.MlgRunInfo(run[0:B].data_ptr(), run[4 * B:5 * B].data_ptr(), run[B:3 * B].data_ptr(),
                        run[3 * B:4 * B].data_ptr(), None, None)
v1 = os.environ.get("MLG_REFIL_ROLLOUT") == "v1"
grid = (B + 1) // 2 + 64  # waves of the two-env kernel (upper bound for the four-env one)
buf = torch.zeros(grid * 32, dtype=torch.int64, device=dev)
_native.call("mlg_refil_debug_set_stamps", _native.ptr(buf))
for i in range(3):
    buf.zero_()
    _native.call("mlg_refil_rollout", _native.byref(spec.to_c()), _native.byref(st.to_c()), _native.byref(ag.dims()),
                 _native.ptr(ag.packed()), _native.byref(mb), _native.byref(ri), 0.05, 0, _native.stream_ptr())
torch.cuda.synchronize()
a = buf.view(grid, 32).cpu().numpy().astype(np.float64)
a = a[a[:, 31] == 1]
grid = len(a)
names = (["ein build", "entity_block (fc1/in_trans/attn)", "post (out/fc2/GRU)", "fc3+select+record", "env exec",
          "env resolve", "env reduce/reward", "hp update + observe", "finish/tails"] if v1 else
         ["loop top", "entity pairs (fc1/in_trans/attn)", "post (out/fc2/GRU)", "fc3+select+onehot", "env exec",
          "env resolve", "env reduce/reward", "hp update + observe", "finish/tails"])
tot = a[:, 30].mean()
print(f"waves={grid} mean cycles/wave={tot:.0f} (s_memtime: shader clock)")
for k, n in enumerate(names):
    print(f"{n:34s} share={a[:, k].mean() / tot * 100:6.1f}%")
if not v1:
    for k, n in ((16, "  fc1 (inputs, loads, MFMAs)"), (17, "  in_trans (4 stages)"), (18, "  attention (VALU)"),
                 (19, "  out_trans"), (20, "  fc2"), (21, "  GRUCell"), (22, "  fc3 + argmax scan"),
                 (23, "  argmax reduce + eps + record")):
        print(f"{n:34s} share={a[:, k].mean() / tot * 100:6.1f}%")
if not v1:
    # per-step cost by kind (slots 9/10 cycles, 11/12 counts: both pairs running / one pair) and the critical wave
    us = 1.0  # cycles
    for k, n in ((0, "both pairs"), (1, "one pair")):
        c, m = a[:, 9 + k].sum(), a[:, 11 + k].sum()
        print(f"{n:12s} steps/wave={m / grid:6.1f}  cyc/step={c / max(m, 1) * us:7.2f}")
    w = int(np.argmax(a[:, 30]))
    print(f"critical wave: total={a[w, 30] * us:.0f} cyc  both={a[w, 11]:.0f} steps x {a[w, 9] / max(a[w, 11], 1) * us:.0f} cyc"
          f"  one={a[w, 12]:.0f} steps x {a[w, 10] / max(a[w, 12], 1) * us:.0f} cyc")
    tq = np.percentile(a[:, 30] * us, [50, 90, 99, 100])
    print("wave totals cyc p50/p90/p99/max:", " ".join(f"{x:.1f}" for x in tq))
    st = a[:, 11] + a[:, 12]
    print("wave steps p50/p90/max:", np.percentile(st, 50), np.percentile(st, 90), st.max())
