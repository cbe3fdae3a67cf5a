"""Times mlg_refil_rollout alone (4096 envs, refil_8, episode_limit 100) with HIP events."""
import os
import sys

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
a = refil_args()
torch.manual_seed(0)
ag = REGISTRY["imagine_entity_attend_rnn"](29, a).to(dev)
scheme, groups, pre = entity_scheme_for(spec.env_info(), torch)
batch = EpisodeBatch(scheme, groups, B, 101, preprocess=pre, device=dev)
mb, keep = mlg_entity_batch(batch)
mb.full_write = 1
st = VecEnvState(spec, B, dev)
run = torch.zeros(6 * B, dtype=torch.int32, device=dev)
ri = _native.MlgRunInfo(run[0:B].data_ptr(), run[4 * B:5 * B].data_ptr(), run[B:3 * B].data_ptr(),
                        run[3 * B:4 * B].data_ptr(), None, None)
cs = spec.to_c()
times, steps = [], []
for i in range(8):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _native.call("mlg_refil_rollout", _native.byref(cs), _native.byref(st.to_c()), _native.byref(ag.dims()),
                 _native.ptr(ag.packed()), _native.byref(mb), _native.byref(ri), 0.05, 0, _native.stream_ptr())
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1))
    steps.append(int(run[0:B].sum()))
ms = sum(times[2:]) / len(times[2:])
n = sum(steps[2:]) / len(steps[2:])
print(f"refil rollout B={B}: {ms:.3f} ms/launch, {n / B:.1f} steps/env, {n / ms * 1e3 / 1e6:.2f} M env-steps/s "
      f"(rollout only); times {['%.2f' % t for t in times]}")
