import os, sys
sys.path[:0] = ["ma-league_amd", "tests", "oracle"]
import numpy as np, torch
from helpers import ref_envs_for
from maleague.custom_logging import MainLogger
from maleague.runs import MultiAgentExperiment
from maleague.utils.config import build_config, to_args
cfg = build_config("qmix", "ma", overrides=["runner=episode", "batch_size_run=1", "buffer_cpu_only=False",
                                            "buffer_size=64", "batch_size=4", "env_args.match_build_plan=small",
                                            "env_args.episode_limit=40", "t_max=1000000",
                                            "test_interval=100000000", "seed=3"])
args = to_args(cfg)
exp = MultiAgentExperiment(args, MainLogger())
st = exp.stepper
print("spec", st.spec.team, st.spec.role, st.spec.melee, st.spec.scripted, st.spec.seed, st.spec.stochastic, st.spec.grid)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
exp.start(max_iterations=n)
torch.cuda.synchronize()
nb = {k: v[:n].detach().cpu().numpy() for k, v in exp.home_buffer.data.transition_data.items()}
ref = ref_envs_for(st.spec, 1, seed=st.spec.seed)[0]
print("t_env", st.t_env, "episodes", exp.home_buffer.episodes_in_buffer, "filled", nb["filled"][:, :, 0].sum(1))
refs = []
r2 = ref_envs_for(st.spec, 1, seed=st.spec.seed)[0]
for k in range(3 * n):
    r2.reset()
    refs.append(r2.state().copy())
for e in range(n):
    m = [k for k in range(3 * n) if np.array_equal(nb["state"][e, 0], refs[k])]
    print(e, "matches oracle episode", m, "st.episode", st.envs.episode.cpu().numpy())
