"""Host time per training iteration of config 2 (launch-side Python + ctypes), measured without syncs, next to the
GPU time per iteration: the loop is host-bound when the first approaches the second."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ma-league_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from maleague.custom_logging import MainLogger  # noqa: E402
from maleague.runs import MultiAgentExperiment  # noqa: E402


class A:
    plan, envs, episode_limit = None, 4096, 100


args, _ = bench.make_args(os.environ.get("MODE", "ai"), A, 0, 0)  # MODE=refil: config 5
exp = MultiAgentExperiment(args, MainLogger(log_interval=10 ** 12))
exp._init_stepper()
st = exp.stepper
st.t_env = 10 ** 6
B = st.batch_size
ep = [0]


def it():  # one iteration of MultiAgentExperiment.start's loop, as bench.py runs it
    ep[0] = exp._iteration(ep[0])


# time the host spends blocked on the summary ring (Event.synchronize: the GPU is behind) is not host work
_wait = [0.0]
_sync = torch.cuda.Event.synchronize


def _timed_sync(self):
    w0 = time.perf_counter()
    _sync(self)
    _wait[0] += time.perf_counter() - w0


torch.cuda.Event.synchronize = _timed_sync
for i in range(5):
    it()
torch.cuda.synchronize()
_wait[0] = 0.0
host = []
t0 = time.perf_counter()
for i in range(20):
    h0 = time.perf_counter()
    it()
    host.append(time.perf_counter() - h0)
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
host.sort()
print(f"host per iteration: median {host[10] * 1e3:.3f} ms, max {host[-1] * 1e3:.3f} ms; host loop {t_host / 20 * 1e3:.3f} "
      f"ms/it; wall incl. GPU {t_all / 20 * 1e3:.3f} ms/it")
print(f"host WORK per iteration (host loop minus the waits on the summary ring): "
      f"{(t_host - _wait[0]) / 20 * 1e3:.3f} ms/it (waits {_wait[0] / 20 * 1e3:.3f} ms/it)")

if os.environ.get("PROFILE"):
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for i in range(20):
        it()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)

buf = exp.home_buffer
tf = [int(buf.sample(args.batch_size, view=True).max_t_filled()) for _ in range(10)]
print(f"sampled batches' filled length (max over the batch's episodes): mean {sum(tf) / len(tf):.1f}, {tf}")
