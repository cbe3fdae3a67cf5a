"""Per-phase cycle breakdown of the learner recurrences (agent_rec4_kernel = 0, agent_bwd4_kernel = 1) from the
diagnostic stamps library (make -C ma-league_amd stamps): runs scripts/bench_learner.py's setup, one stamped
train() call, and prints mean cycles per step of each phase over the waves of valid blocks."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MLG_LIB"] = os.path.join(ROOT, "ma-league_amd", "maleague", "_lib", "libmaleague_stamps.so")
os.environ.setdefault("REPS", "3")
sys.argv = [sys.argv[0]]
g = runpy.run_path(os.path.join(ROOT, "scripts", "bench_learner.py"))
import torch
from maleague import _native

buf = torch.zeros(2 * 1024 * 8 * 8, dtype=torch.int64, device="cuda")
_native.call("mlg_debug_set_learner_stamps", _native.ptr(buf))
g["lrn"].train(g["samples"][0], 10 ** 6, 0)
torch.cuda.synchronize()
st = buf.view(2, 1024, 8, 8).cpu()
names = {0: ["mfma+xchg", "refill", "cell+lds_w", "stores", "barrier", "prologue"],
         1: ["lds_r+mfma+xchg", "loads+coef", "dh*coef+lds_w", "stores", "barrier", "prologue"]}
for kid, kname in [(0, "rec4"), (1, "bwd4")]:
    s = st[kid].reshape(-1, 8)
    s = s[s[:, 6] > 0].double()
    steps = s[:, 6].mean().item()
    print(f"{kname}: waves={len(s)} steps={steps:.0f} total_cycles={s[:, 7].mean().item():.0f} "
          f"per_step={s[:, 7].mean().item() / steps:.0f}")
    for k, nm in enumerate(names[kid]):
        per = s[:, k].mean().item() / (1 if k == 5 else steps)
        print(f"   {nm:18s} {per:9.1f} cycles{'' if k == 5 else '/step'}  (min {s[:, k].min().item() / (1 if k == 5 else steps):.0f}"
              f" max {s[:, k].max().item() / (1 if k == 5 else steps):.0f})")
