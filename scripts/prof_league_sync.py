"""Host profile of the league exchange (LeagueInstance.sync) as bench.py's league leg runs it at N=1: the wall time
of each sync after a drained training iteration, and a cProfile of ten of them. GPU box only."""
import cProfile
import os
import pstats
import sys
import time
import types

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "ma-league_amd"), ROOT]

import torch  # noqa: E402

import bench  # noqa: E402
from maleague.custom_logging import MainLogger  # noqa: E402
from maleague.league import DistributedLeague, LeagueInstance  # noqa: E402

a = types.SimpleNamespace(envs=4096, episode_limit=100, plan=None)
args, _ = bench.make_args("league", a, 0, 0)
lg = DistributedLeague(n_players=1, device=torch.device("cuda:0"), seed=0, max_historical=4)
if os.environ.get("MODE", "bench") == "bench":  # the bench's N = 1 league (AlphaStar roles, bench.league_setup)
    lmode, roles = bench.league_setup(1, args)
    inst = LeagueInstance(args, MainLogger(log_interval=10 ** 12), lg, mode=lmode, role=roles, seed=0)
else:
    inst = LeagueInstance(args, MainLogger(log_interval=10 ** 12), lg, mode="matchmaking", seed=0)
inst.experiment.stepper.t_env = 10 ** 6
for _ in range(3):
    inst.sync()
    inst.play(1)
torch.cuda.synchronize()
ts = []
for _ in range(5):  # unprofiled
    inst.play(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    inst.sync()
    ts.append(time.perf_counter() - t0)
print("sync ms (no profiler):", [round(t * 1e3, 3) for t in ts], flush=True)
ts = []
pr = cProfile.Profile()
for _ in range(int(os.environ.get("SYNCS", "10"))):
    inst.play(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pr.enable()
    inst.sync()
    pr.disable()
    ts.append(time.perf_counter() - t0)
print("sync ms (cProfile):", [round(t * 1e3, 3) for t in ts], flush=True)
st = pstats.Stats(pr).stats
n = len(ts)
print("us per sync: cumulative, own, calls, function")
for (f, line, name), (cc, nc, tt, ct, _) in sorted(st.items(), key=lambda kv: -kv[1][3])[:45]:
    print(f"{ct / n * 1e6:9.1f} {tt / n * 1e6:9.1f} {nc / n:6.1f}  {os.path.basename(f)}:{line}({name})")
