"""Debug helper: per-parameter gradient comparison of mlg_qlearner_train vs the oracle (autograd)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ma-league_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

import learner_ref as LR
from helpers import qmix_args
from test_gpu_learner import _learner

name = sys.argv[1] if len(sys.argv) > 1 else "qlearner_qmix_dq.npz"
d = np.load(os.path.join(ROOT, "tests", "golden", name))
args = qmix_args()
dev = torch.device("cuda:0")
learner, eb, log = _learner(d, dev, args)
ref = LR.QLearnerRef({k[9:]: d[k] for k in d.files if k.startswith("p0.agent.")},
                     {k[9:]: d[k] for k in d.files if k.startswith("p0.mixer.")}, args)
# oracle grads (pre-clip): replicate train up to backward
b = LR.batch_from_npz(d)
ref.opt.step = lambda *a, **k: None
orig = torch.nn.utils.clip_grad_norm_
norms = {}
def fake_clip(params, max_norm):
    grads = [p.grad.detach().clone() for p in params]
    norms["pre"] = grads
    return orig(params, max_norm)
torch.nn.utils.clip_grad_norm_ = fake_clip
st = ref.train(b, 100, 0)
torch.nn.utils.clip_grad_norm_ = orig
learner.train(eb, 100, 0)
coef = min(10.0 / (learner.last_stats["grad_norm"] + 1e-6), 1.0)
print("stats gpu", learner.last_stats)
print("stats ref", st)
names = list(ref.p.keys()) + ["mixer." + k for k in ref.mp.keys()]
for (p, off, k), g_ref, nm in zip(learner._flat.views, norms["pre"], names):
    g = (learner._grads[off:off + k].cpu().view_as(g_ref) / coef)
    err = (g - g_ref).abs().max().item()
    print(f"{nm:28s} |g|={g_ref.norm():10.5f} maxabs={g_ref.abs().max():10.5f} err={err:.3e} "
          f"rel={err / (g_ref.abs().max().item() + 1e-12):.2e}")
