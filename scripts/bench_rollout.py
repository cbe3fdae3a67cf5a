"""Deterministic rollout-kernel microbenchmark: fixed random policy, the same episodes every repetition
(env episode counters reset), 4096 envs, medium_1h_4t, episode_limit 100, epsilon 0.05. RING=1: train-mode runs
write into a 5000-episode replay ring in full-write mode (the bench's path); each run is inserted.
Prints mean kernel ms (HIP events) per kernel variant given in MLG_BENCH_KERNELS (default "v2")."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ma-league_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch

from helpers import qmix_args, scheme_for
from maleague.components.episode_batch import EpisodeBatch
from maleague.controllers import BasicMAC
from maleague.custom_logging import MainLogger
from maleague.envs.teams_env import VecEnvState
from maleague.steppers import ParallelStepper

B = int(os.environ.get("ENVS", "4096"))
REPS = int(os.environ.get("REPS", "10"))
args = qmix_args(batch_size_run=B, seed=0, env_args={"match_build_plan": os.environ.get("PLAN", "medium_1h_4t"),
                                                     "grid_size": 20, "stochastic_spawns": True, "episode_limit": 100})
stepper = ParallelStepper(args, MainLogger())
info = stepper.get_env_info()
args.n_agents, args.n_actions, args.state_shape = info["n_agents"], info["n_actions"], info["state_shape"]
scheme, groups, preprocess = scheme_for(info, torch)
proto = EpisodeBatch(scheme, groups, 1, 2, preprocess=preprocess, device="cuda")
torch.manual_seed(0)
mac = BasicMAC(proto.scheme, groups, args)
stepper.initialize(scheme, groups, preprocess, mac)
ring = None
if int(os.environ.get("RING", "0")):
    from maleague.components.replay_buffer import ReplayBuffer
    ring = ReplayBuffer(scheme, groups, 5000, 101, preprocess=preprocess, device="cuda")
    assert stepper.attach_replay(ring)
out = {}
for k in os.environ.get("MLG_BENCH_KERNELS", "v7").split(","):
    os.environ["MLG_ROLLOUT_KERNEL"] = k
    ms = []
    for r in range(REPS + 2):
        stepper.envs = VecEnvState(stepper.spec, B, "cuda")
        stepper.t_env = 10 ** 6
        stepper.timing = []
        stepper.run(test_mode=bool(int(os.environ.get("TEST_MODE", "0"))))
        if ring is not None:
            ring.insert_episode_batch(stepper.home_batch)
        torch.cuda.synchronize()
        if r >= 2:
            ms.append(stepper.timing[0][0].elapsed_time(stepper.timing[0][1]))
    lens = stepper.last_run["ep_len"].numpy()
    b = stepper.home_batch
    fil = b["filled"][:, :, 0].bool()
    dead = (b["avail_actions"][:, :, :, 0] == 1) & fil[:, :, None]
    out[k + "_dead_agent_frac"] = float(dead.sum()) / float(fil.sum() * args.n_agents)
    out[k] = {"kernel_ms": sum(ms) / len(ms), "min_ms": min(ms), "env_steps": int(lens.sum()),
              "mean_len": float(lens.mean())}
print(json.dumps(out))
