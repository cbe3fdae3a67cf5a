"""bench.py -- env-steps/sec (rollout + learn), 5v5 QMIX, 4096 envs per GPU (BASELINE.json configs 2-4).

One "step" = one training iteration of a learner: one batched rollout launch over its 4096 envs + insert into
the HBM replay buffer + one QLearner.train on 32 sampled episodes (MultiAgentExperiment._train_episode,
src/runs/train/ma_experiment.py:224-241). value = env steps (t_env increments, parallel_stepper.py:178-179)
of all ranks / max-over-ranks time.

Modes (--mode auto = ai at every N: the metric's config-2 workload per GPU, weak scaling):
  ai        config 2: one learner vs the scripted AI per GPU; N > 1 = N independent learners (one per GPU,
            4096 envs each, no data-path collective: learners never exchange anything on the rollout/learn path)
  refil     config 5: REFIL (entity-attention agent, imagined groups, FlexQMixer), 3-8 agents per env padded to 8,
            4096 envs per GPU vs the scripted AI (entity env variant); N > 1 = independent replicas
  league    config 3 (N = 2: two PFSP self-play learners, opponent swap over RCCL) / config 4 (N >= 4:
            AlphaStar roles, half main players, half main exploiters, historical snapshots): one league player
            per GPU; every --match-len iterations a league iteration exchanges parameters (all_gather) and
            payoff (all_reduce) over RCCL and picks the next opponent. Works at N = 1 too (the player faces
            its own snapshots): the per-GPU cost of a league learner.
N > 1: one process per GPU (torch.distributed.run); rollouts and learners never cross GPUs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "ma-league_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

FP32_MFMA_PEAK = 157.3e12  # MI355X dense fp32 (MFMA == VALU rate), MI355X_MICROARCH.md chip table
HBM_PEAK = 8.0e12


def agent_flops_per_forward(N, d_in, H, A):
    """Algorithmic FLOPs of one BasicMAC.forward per env (drqn_agent.py:29-35 for N agents)."""
    return N * 2 * (d_in * H + 2 * H * 3 * H + H * A)


def refil_flops_per_forward(NA, NE, D0, E, H, A, heads=4):
    """Algorithmic FLOPs of one EntityMAC step per env (entity_rnn_agent.py:32-65 on padded tensors): fc1 and
    in_trans over all entities, attention for the agent queries, out_trans / fc2 / GRUCell / fc3 per agent."""
    hd = E // heads
    att = 2 * heads * NA * NE * hd * 2
    return (2 * NE * D0 * E + 2 * NE * E * 3 * E + att + 2 * NA * E * E * 2 + NA * 2 * (2 * H * 3 * H)
            + 2 * NA * H * A)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="auto", choices=["auto", "ai", "league", "refil"])
    ap.add_argument("--match-len", type=int, default=5, help="league: training iterations per league iteration")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo for rehearsals)")
    ap.add_argument("--device", type=int, default=None, help="GPU index for every rank (rehearsal on one GPU)")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--episode-limit", type=int, default=100)
    ap.add_argument("--plan", default=None, help="match_build_plan (default medium_1h_4t; refil: refil_8)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per rollout launch (scripts/gpu_traffic.sh -> profiles/)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.device is not None:
        local_rank = a.device
    mode = a.mode if a.mode != "auto" else "ai"
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
        else:
            dist.init_process_group(a.backend)
    dev = torch.device(f"cuda:{local_rank}")
    torch.cuda.set_device(dev)

    from maleague.custom_logging import MainLogger
    from maleague.runs import MultiAgentExperiment
    from maleague.utils.config import build_config, to_args

    plan = a.plan or ("refil_8" if mode == "refil" else "medium_1h_4t")
    overrides = [f"batch_size_run={a.envs}", "runner=parallel", "buffer_cpu_only=False",
                 f"env_args.match_build_plan={plan}", f"env_args.episode_limit={a.episode_limit}",
                 f"seed={rank}", "learner_log_interval=1000000000", "log_interval=1000000000",
                 "runner_log_interval=1000000000", "test_interval=1000000000000", "t_max=1000000000000",
                 "show_exp_parameters=False", "league_checkpoint_min_steps=20000", "league_checkpoint_max_steps=40000"]
    if mode == "refil":
        cfg = build_config("refil", "ma_entity", overrides=overrides, device_index=local_rank)
    else:
        cfg = build_config("qmix", "ma", overrides=overrides, device_index=local_rank)
    import numpy as np
    np.random.seed(rank)  # replay sampling (reproducible learning curve -> reproducible episode lengths)
    torch.manual_seed(rank)
    args = to_args(cfg)
    inst = None
    if mode in ("ai", "refil"):
        exp = MultiAgentExperiment(args, MainLogger(log_interval=10 ** 12))
        exp._init_stepper()
        if mode == "refil":
            ea = args.env_args
            workload = (f"refil_{plan}_{ea.get('min_agents', 3)}to{ea.get('max_agents', 8)}agents_{a.envs}envs_"
                        f"ep{a.episode_limit}")
            parallelism = f"replicas{world}"
        else:
            workload = f"qmix_5v5_{plan}_{a.envs}envs_ep{a.episode_limit}"
            parallelism = f"replicas{world}"
    else:
        from maleague.league import DistributedLeague, LeagueInstance, league_roles_for
        lg = DistributedLeague(n_players=world, device=dev, seed=0, max_historical=8 * world)
        if world >= 4:
            roles = league_roles_for(world, args)
            inst = LeagueInstance(args, MainLogger(log_interval=10 ** 12), lg, mode="rolebased", role=roles, seed=0)
            n_main = roles.count("main")
            workload = f"pfsp_league_{n_main}main_{world - n_main}exploiter_qmix_5v5_{plan}_{a.envs}envs_ep{a.episode_limit}"
        else:
            inst = LeagueInstance(args, MainLogger(log_interval=10 ** 12), lg, mode="matchmaking", seed=0)
            workload = f"selfplay_pfsp_{world}learners_qmix_5v5_{plan}_{a.envs}envs_ep{a.episode_limit}"
        exp = inst.experiment
        parallelism = f"league{world}_rccl"
    stepper = exp.stepper
    B = stepper.batch_size
    # steady-state exploration (epsilon floor 0.05), as SURVEY §8d prescribes for timing runs
    stepper.t_env = 10 ** 6
    episode = 0

    def iteration(i):
        nonlocal episode
        if inst is None:
            exp._train_episode(episode)
            episode += B
        else:
            if i % a.match_len == 0:
                inst.sync()  # league iteration: payoff all_reduce + parameter all_gather over RCCL, next match
            inst.play(1)

    for i in range(a.warmup):
        iteration(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    # rollout-kernel timing with HIP events on the stream the kernel is launched on
    stepper.timing = []
    t0_env = stepper.t_env
    rows0 = int(stepper.agent_rows.item())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        iteration(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    env_steps = stepper.t_env - t0_env
    local_env_steps = env_steps
    rows_per_launch = (int(stepper.agent_rows.item()) - rows0) / a.steps
    if dist:
        rdev = dev if a.backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([env_steps], dtype=torch.float64, device=rdev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        env_steps = int(s.item())
    ev_ms = [st.elapsed_time(en) for st, en in stepper.timing]
    stepper.timing = None
    value = env_steps / elapsed

    # roofline of the dominant kernel (the rollout): fp32 MFMA-bound agent cell
    info = stepper.get_env_info()
    sides = 2 if mode == "league" else 1
    N, A = info["n_agents"] // sides, info["n_actions"]
    if mode == "refil":
        fl = refil_flops_per_forward(N, info["n_entities"], info["entity_shape"] + A, 64, 64, A)
    else:
        d_in = info["obs_shape"] + A + N
        fl = sides * agent_flops_per_forward(N, d_in, 64, A)
    # agent forwards per launch: every env steps len times and records one final action (len + 1 forwards)
    forwards = (local_env_steps + a.steps * B) / a.steps
    avg_kernel_s = sum(ev_ms) / len(ev_ms) / 1e3
    achieved = fl * forwards / avg_kernel_s
    issued = fl / (sides * N) * rows_per_launch / avg_kernel_s if mode == "ai" else None
    traffic = None
    kc1 = (info.get("entity_shape", 0) + A + 15) // 16 if mode == "refil" else 0
    # the default rollout kernel: v7 (split-bf16 GRU), compile-time shape for the 5v5 / 3v3 plans
    v7 = "rollout_v2_kernel<64, true, 5, 10>" if (N, info["n_actions"]) == (5, 15) else (
        "rollout_v2_kernel<64, true, 3, 6>" if (N, info["n_actions"]) == (3, 11) else "rollout_v2_kernel<64, true>")
    sp7 = "rollout_sp7_kernel<10, 10>" if (N, info["n_actions"]) == (5, 15) else (
        "rollout_sp7_kernel<6, 6>" if (N, info["n_actions"]) == (3, 11) else "rollout_sp7_kernel<0, 0>")
    kernel = {"ai": v7, "league": sp7,  # the bench runs H = 64 (rnn_hidden_dim below)
              "refil": f"refil_rollout_kernel<{kc1}>"}[mode]
    if a.traffic_json and os.path.exists(a.traffic_json):
        with open(a.traffic_json) as f:
            traffic = json.load(f).get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")

    cpu = None
    if rank == 0 and world == 1 and mode in ("ai", "refil") and not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cpu_baseline
        threads = min(16, os.cpu_count() or 1)
        if mode == "refil":
            r = cpu_baseline.run_refil(seconds=a.cpu_seconds, B=32, episode_limit=a.episode_limit, threads=threads)
            what = "C entity env + PyTorch-CPU EntityAttentionRNNAgent / REFILLearner (refil_ref)"
        else:
            r = cpu_baseline.run(seconds=a.cpu_seconds, B=64, episode_limit=a.episode_limit, threads=threads)
            what = "oracle stepper + C env + PyTorch-CPU DRQN/QMIX learner"
        cpu = {"value": r["value"], "unit": "env-steps/s", "cores": r["cores"], "kind": "port",
               "sample": f"{r['runs']} runs x {r['B']} envs (+1 train each), {r['env_steps']} env steps in "
                         f"{r['seconds']:.1f}s; {what}"}
    if rank == 0:
        out = {"metric": "env-steps/sec (rollout+learn), 5v5 QMIX, 4096 envs, at 1/2/4/8 MI355X",
               "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
               "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "f32",
               "data": ("synthetic (entity battles, 3-8 agents per env padded to 8, random-init REFIL)"
                        if mode == "refil" else "synthetic (spec-v1 5v5 battles, random-init QMIX)"),
               "config": {"workload": workload, "mode": mode, "envs_per_gpu": B, "episode_limit": a.episode_limit,
                          "learner_batch": 32, "rnn_hidden_dim": 64, "buffer_size": 5000,
                          "parallelism": parallelism, **({"match_len": a.match_len} if inst else {})},
               "env_steps": env_steps, "mean_episode_len": env_steps / max(1, a.steps * B * world),
               "roofline": {"bound": "mfma", "achieved": achieved / 1e12, "peak": FP32_MFMA_PEAK / 1e12,
                            "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK, "traffic": traffic,
                            "kernel": kernel, "avg_kernel_ms": avg_kernel_s * 1e3,
                            "flops_per_launch": fl * forwards},
               "cpu_baseline": cpu}
        if issued is not None:
            out["roofline"].update({"issued_tflops": issued / 1e12, "issued_frac": issued / FP32_MFMA_PEAK,
                                    "issued_rows_per_launch": rows_per_launch})
        if mode == "ai" and kernel.startswith("rollout_v2_kernel<64, true"):
            out["roofline"]["note"] = ("fp32 algorithmic FLOPs vs the fp32 MFMA peak; the GRU products run as "
                                       "split-bf16 fp32 emulation (6 bf16 MFMA partial products each, DESIGN.md §4a)")
        if inst is not None:
            out["league"] = {"opponents_rank0": [h[1] for h in inst.history],
                             "historical_snapshots": len(inst.league.historical_meta)}
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
