"""bench.py -- env-steps/sec (rollout + learn), 5v5 QMIX, 4096 envs per GPU (BASELINE.json configs 2-5).

One "step" = one training iteration of a learner: one batched rollout launch over its 4096 envs + insert into
the HBM replay buffer + one QLearner.train on 32 sampled episodes (MultiAgentExperiment._train_episode,
src/runs/train/ma_experiment.py:224-241). value = env steps (t_env increments, parallel_stepper.py:178-179)
of all ranks / max-over-ranks time.

Modes:
  auto      (default) two legs in one run, both at every N:
            * ``value`` = config 2 per GPU: one learner vs the scripted AI on every rank (N independent learners,
              no data-path collective; weak scaling) -- the metric's "5v5 QMIX, 4096 envs, at 1/2/4/8 MI355X";
            * ``league`` = the league at the same N: config 3 at N = 2 (two PFSP self-play learners, opponent swap
              over RCCL), config 4 at N >= 4 (AlphaStar roles: half main players, half main exploiters, historical
              snapshots), at N = 1 one league player facing its own snapshots (the per-GPU cost of a league
              learner, the denominator of the league's scaling). The league exchange (payoff all_reduce,
              parameter all_gather, barrier, matchmaking) runs every --match-len iterations INSIDE the timed
              region; its wall time is reported (exchange_ms_*).
  ai        config 2 only
  league    the league leg only (as ``value``)
  refil     config 5: REFIL (entity-attention agent, imagined groups, FlexQMixer), 3-8 agents per env padded to
            8, 4096 envs per GPU vs the scripted AI (entity env variant); N > 1 = replicas
N > 1: one process per GPU (torch.distributed.run, RCCL); rollouts and learners never cross GPUs. Under
torch.distributed.run with one process the league's collectives still run (RCCL at world size 1).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "ma-league_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402

FP32_MFMA_PEAK = 157.3e12  # MI355X dense fp32 (MFMA == VALU rate), MI355X_MICROARCH.md chip table
HBM_PEAK = 8.0e12
CLOCK_HZ = 2.4e9  # MI355X max engine clock (MI355X_MICROARCH.md): the latency floor is a lower bound
# HIP-event pair around every k-th rollout launch of the timed region (--timing-every). Every launch (default): the
# pair costs ~8-10 us of queue time per iteration (0.7 % of ms_per_step at config 2, a device-scope-release event
# pair the same), but a sample of every 4th launch biases the kernel average (launch times vary 0.68-1.03 ms with
# the iteration's longest episode): profiles/r04/s11_timing_ab/
TIMING_EVERY = 1
LEAGUE_CKPT_STEPS = 8000
METRIC = "env-steps/sec (rollout+learn), 5v5 QMIX, 4096 envs, at 1/2/4/8 MI355X"
COUNTERS_JSON = os.path.join(ROOT, "profiles", "counters.json")


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


# ---- distributed plumbing ----------------------------------------------------------------------------------
class Ctx:
    """Where this rank runs: torch.distributed (or not), its device, where reductions stage their tensors."""

    def __init__(self, dist, dev):
        self.dist, self.dev = dist, dev
        self.world = dist.get_world_size() if dist else 1
        self.rank = dist.get_rank() if dist else 0
        self.rdev = dev if (dist and dist.get_backend() == "nccl") else torch.device("cpu")

    def sync(self):
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def reduce(self, x: float, op: str) -> float:
        if not self.dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.rdev)
        self.dist.all_reduce(t, op={"max": self.dist.ReduceOp.MAX, "sum": self.dist.ReduceOp.SUM}[op])
        return float(t.item())

    def gather(self, x: float) -> list:
        if not self.dist:
            return [x]
        t = torch.tensor([x], dtype=torch.float64, device=self.rdev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [float(o.item()) for o in out]


def timed_loop(ctx: Ctx, iteration, stepper, steps: int, warmup: int) -> dict:
    """W untimed iterations, then exactly K timed ones bracketed by barrier + device sync on both sides.
    Rollout launches inside the timed region are timed with HIP events on their own stream (stepper.timing)."""
    for i in range(warmup):
        iteration(i)
    ctx.sync()
    ctx.barrier()
    timing_ok = ctx.dev.type == "cuda"
    stepper.timing = [] if timing_ok else None
    stepper.timing_every = TIMING_EVERY if steps >= 2 * TIMING_EVERY else 1  # short runs: every launch
    stepper._launches = 0  # sampled launches counted from the start of the timed region
    t0_env = stepper.t_env
    run0 = stepper._run_id  # runs launched from here on are the timed ones
    stepper.t_history = []
    rows0 = int(stepper.agent_rows.item())
    ctx.sync()
    t0 = time.perf_counter()
    for i in range(steps):
        iteration(i)
    ctx.sync()
    ctx.barrier()
    elapsed_local = time.perf_counter() - t0
    local_steps = stepper.t_env - t0_env
    longest = [t for rid, t in stepper.t_history if rid > run0]
    stepper.t_history = None
    rows = (int(stepper.agent_rows.item()) - rows0) / steps
    ev_ms = [st.elapsed_time(en) for st, en in stepper.timing] if timing_ok else []
    stepper.timing = None
    elapsed = ctx.reduce(elapsed_local, "max")
    per_rank = ctx.gather(local_steps / elapsed_local)
    total = int(ctx.reduce(float(local_steps), "sum"))
    return {"elapsed": elapsed, "env_steps": total, "local_env_steps": local_steps, "per_rank": per_rank,
            "value": total / elapsed, "ms_per_step": elapsed / steps * 1e3, "rows_per_launch": rows,
            "avg_kernel_ms": (sum(ev_ms) / len(ev_ms)) if ev_ms else None,
            "longest_episode_mean": (sum(longest) / len(longest)) if longest else None}


def league_iteration(inst, match_len: int, exchange_s: list, ctx=None):
    """One training iteration of a league player; every ``match_len`` iterations a league iteration first
    (LeagueInstance.sync: payoff all_reduce, parameter / checkpoint all_gather, barrier, matchmaking --
    matchmaking_league_instance.py:36-68), its wall time appended to ``exchange_s``. The exchange reads the
    replicated state on the host, so it drains this rank's queued iterations first; the drain is excluded from
    the exchange's time (it is training time), the wait for the other ranks is not."""

    def it(i):
        if i % match_len == 0:
            if ctx is not None:
                ctx.sync()
            t0 = time.perf_counter()
            inst.sync()
            exchange_s.append(time.perf_counter() - t0)
        inst.play(1)

    return it


def run_league_leg(ctx: Ctx, inst, steps: int, warmup: int, match_len: int) -> dict:
    """The league leg of the bench (also driven by tests/test_bench_league.py over gloo on CPU). The warm-up runs at
    least match_len + 1 iterations, so it holds a league iteration after some training (the first snapshot)."""
    warmup = max(warmup, match_len + 1)
    ex_warm, ex = [], []
    warm_it = league_iteration(inst, match_len, ex_warm, ctx)
    timed_it = league_iteration(inst, match_len, ex, ctx)
    n = [0]

    def it(i):
        (warm_it if n[0] < warmup else timed_it)(i)
        n[0] += 1

    r = timed_loop(ctx, it, inst.experiment.stepper, steps, warmup)
    ex_ms = [e * 1e3 for e in ex]
    lg = inst.league
    r.update({"league_iterations": len(ex), "league_warmup_iterations": warmup, "exchange_ms_mean": sum(ex_ms) / max(1, len(ex_ms)),
              "exchange_ms_max": max(ex_ms) if ex_ms else None,
              "exchange_frac": sum(ex) / r["elapsed"] if r["elapsed"] > 0 else None,
              "collective_backend": lg.backend, "world_size": ctx.world,
              "opponents_rank0": [h[1] for h in inst.history], "historical_snapshots": len(lg.historical_meta),
              "snapshots_taken": len(lg.historical_meta) + lg.evictions,
              "historical_matches_rank0": sum(1 for h in inst.history if h[2]),
              "historical_matches_timed_rank0": sum(1 for h in inst.history[-len(ex):] if h[2]) if ex else 0,
              "evictions": lg.evictions,
              "payoff_games": float(lg.payoff.tensor[..., 0].sum().item()),
              "teams": ([t.codes() for t in inst.teams] if getattr(inst, "teams", None) is not None else None),
              "away_teams_rank0": sorted(set(getattr(inst, "away_teams", None) or [])) or None})
    return r


# ---- experiments ---------------------------------------------------------------------------------------------
def make_args(mode, a, rank, local_rank):
    from maleague.utils.config import build_config, to_args
    plan = a.plan or ("refil_8" if mode == "refil" else "medium_1h_4t")
    overrides = [f"batch_size_run={a.envs}", "runner=parallel", "buffer_cpu_only=False",
                 f"env_args.match_build_plan={plan}", f"env_args.episode_limit={a.episode_limit}",
                 f"seed={rank}", "learner_log_interval=1000000000", "log_interval=1000000000",
                 "runner_log_interval=1000000000", "test_interval=1000000000000", "t_max=1000000000000",
                 "show_exp_parameters=False",
                 # a snapshot after every ~3 train calls (a 32-episode batch trains on <= 3.2 k env steps): the first
                 # fires in the league leg's warm-up, the timed league iterations then gather snapshots and play
                 # historical opponents (the reference's 2e9 / 4e9 would never fire in a bench)
                 f"league_checkpoint_min_steps={LEAGUE_CKPT_STEPS}", f"league_checkpoint_max_steps={LEAGUE_CKPT_STEPS}"]
    if mode == "refil":
        cfg = build_config("refil", "ma_entity", overrides=overrides, device_index=local_rank)
    else:
        cfg = build_config("qmix", "ma", overrides=overrides, device_index=local_rank)
    import numpy as np
    np.random.seed(rank)  # replay sampling (reproducible learning curve -> reproducible episode lengths)
    torch.manual_seed(rank)
    return to_args(cfg), plan


def league_setup(world: int, args):
    """(mode, roles) of the league leg at ``world`` ranks. Every N runs AlphaStar roles, so every player takes
    historical snapshots (main_player.py:120-132) and plays them (PFSP over historical, :33-35): N = 1 one main
    player against its own snapshots, N = 2 (config 3) two main players (self-play + PFSP over the pool), N >= 4
    (config 4) main players + main exploiters (league_roles_for)."""
    from maleague.league import league_roles_for
    if world >= 4:
        return "rolebased", league_roles_for(world, args)
    return "rolebased", ["main"] * world


def league_teams(world: int, a):
    """Every league player's team (central_worker.py:44-50, 84-93): ``n_teams`` compositions sampled by the
    TeamComposer with the forced unit (force-unit --role HEALER --attack RANGED, unique, sorted first), one per
    main player; at N >= 4 each team fields a main player and a main exploiter (alpha_star_league.py:23-40: player p
    and p + N/2 share team p). ``--league-teams mirror``: every player plays the env plan mirrored (round 5)."""
    if a.league_teams == "mirror":
        return None, 0
    from maleague.league.teams import compose_league_teams
    n_teams = world if world < 4 else world // 2
    teams = compose_league_teams(5, n_teams, "HEALER", "RANGED", unique=True, seed=0)
    return [teams[p % n_teams] for p in range(world)], n_teams


def league_workload(world, plan, a, roles=None, n_teams=0):
    comp = f"composed{n_teams}teams_forceHR" if n_teams else plan
    if world >= 4:
        n_main = roles.count("main")
        return (f"pfsp_league_{n_main}main_{world - n_main}exploiter_qmix_5v5_{comp}_{a.envs}envs_ep{a.episode_limit}",
                "BASELINE config 4 (PFSP league: main players + main exploiters, one composed team per main / exploiter "
                "pair, historical snapshots, RCCL)")
    if world > 1:
        return (f"selfplay_pfsp_{world}learners_qmix_5v5_{comp}_{a.envs}envs_ep{a.episode_limit}",
                f"BASELINE config 3 (self-play QMIX, {world} learners as main players with their own composed teams: "
                f"self-play + PFSP over historical snapshots, opponent swap via RCCL)")
    return (f"league_player_vs_own_snapshots_qmix_5v5_{comp}_{a.envs}envs_ep{a.episode_limit}",
            "1-GPU league player (self-play vs its own snapshots): the per-GPU league cost, scaling denominator")


def kernel_names(mode, N, A, kc1=0):
    v7 = "rollout_v2_kernel<64, true, 5, 10>" if (N, A) == (5, 15) else (
        "rollout_v2_kernel<64, true, 3, 6>" if (N, A) == (3, 11) else "rollout_v2_kernel<64, true>")
    # self-play: the one-round sp8 kernel for the static 5v5 / 3v3 shapes, sp7 otherwise (MLG_ROLLOUT_KERNEL=sp7: sp7)
    sp8_on = os.environ.get("MLG_ROLLOUT_KERNEL") not in ("sp7", "sp2", "v1") and not os.environ.get("MLG_ROLLOUT_GENERIC")
    if sp8_on and (N, A) in ((5, 15), (3, 11)):
        sp7 = "rollout_sp8_kernel<10, 10>" if (N, A) == (5, 15) else "rollout_sp8_kernel<6, 6>"
    else:
        sp7 = "rollout_sp7_kernel<10, 10>" if (N, A) == (5, 15) else (
            "rollout_sp7_kernel<6, 6>" if (N, A) == (3, 11) else "rollout_sp7_kernel<0, 0>")
    # the four-env kernel for the entity width of the env variant; its refil_8 shape (8 agents, 21 actions) runs the
    # static 16-unit instantiation unless MLG_REFIL_GENERIC is set
    st16 = (N, A) == (8, 21) and not os.environ.get("MLG_REFIL_GENERIC")
    refil = (f"refil_rollout_kernel<{kc1}>" if (os.environ.get("MLG_REFIL_ROLLOUT") == "v1" or kc1 != 2)
             else f"refil_rollout4_kernel<2, {16 if st16 else 0}>")
    return {"ai": v7, "league": sp7, "refil": refil}[mode]


def load_counters(kernel):
    """Committed rocprofv3 counter results for ``kernel`` (scripts/gpu_counters.sh -> profiles/counters.json):
    HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction), MFMA-busy fraction
    (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)), wave-parked fraction, profiled commit."""
    if not os.path.exists(COUNTERS_JSON):
        return {}
    with open(COUNTERS_JSON) as f:
        return json.load(f).get("kernels", {}).get(kernel, {})


def roofline(mode, stepper, r, steps, B):
    info = stepper.get_env_info()
    sides = 2 if mode == "league" else 1
    N, A = info["n_agents"] // sides, info["n_actions"]
    kc1 = (info.get("entity_shape", 0) + A + 15) // 16 if mode == "refil" else 0
    if mode == "refil":
        fl = refil_flops_per_forward(N, info["n_entities"], info["entity_shape"] + A, 64, 64, A)
    else:
        fl = sides * agent_flops_per_forward(N, info["obs_shape"] + A + N, 64, A)
    # agent forwards per launch: every env steps len times and records one final action (len + 1 forwards)
    forwards = (r["local_env_steps"] + steps * B) / steps
    if r["avg_kernel_ms"] is None:  # --timing-every 0 (A/B runs): no kernel timing
        return {"bound": "mfma", "achieved": None, "peak": FP32_MFMA_PEAK / 1e12, "unit": "TFLOP/s", "frac": None,
                "traffic": None, "kernel": kernel_names(mode, N, A), "avg_kernel_ms": None}
    avg_s = r["avg_kernel_ms"] / 1e3
    achieved = fl * forwards / avg_s
    kernel = kernel_names(mode, N, A, kc1)
    cnt = load_counters(kernel)
    traffic = cnt.get("hbm_bytes_per_launch")
    out = {"bound": "mfma", "achieved": achieved / 1e12, "peak": FP32_MFMA_PEAK / 1e12, "unit": "TFLOP/s",
           "frac": achieved / FP32_MFMA_PEAK, "traffic": traffic, "kernel": kernel,
           "avg_kernel_ms": r["avg_kernel_ms"], "flops_per_launch": fl * forwards,
           "hbm_gbps": traffic / avg_s / 1e9 if traffic else None,
           "hbm_frac": traffic / avg_s / HBM_PEAK if traffic else None,
           "mfma_busy": cnt.get("mfma_busy"), "wave_parked": cnt.get("wait_any_frac"),
           "counters_commit": cnt.get("commit")}
    # the bound the rollout actually has: a launch lasts at least as long as its longest episode,
    # whose steps are serial (agent step of t feeds the env step of t feeds the agent step of t + 1); each costs at
    # least the measured cycles of a step with that one env running (phase stamps, diagnostic build). The floor:
    # mean over the timed launches of (longest episode + 1 final agent step) x those cycles / the max clock.
    step_cyc = cnt.get("one_env_step_cycles")
    if step_cyc and r.get("longest_episode_mean"):
        floor_ms = (r["longest_episode_mean"] + 1) * step_cyc / CLOCK_HZ * 1e3
        out.update({"latency_floor_ms": floor_ms, "latency_floor_frac": floor_ms / r["avg_kernel_ms"],
                    "one_env_step_cycles": step_cyc, "one_env_step_source": cnt.get("one_env_step_source"),
                    "one_env_step_commit": cnt.get("one_env_step_commit"),
                    "longest_episode_mean": r["longest_episode_mean"], "latency_floor_clock_ghz": CLOCK_HZ / 1e9})
    if mode == "ai":
        issued = fl / N * r["rows_per_launch"] / avg_s
        out.update({"issued_tflops": issued / 1e12, "issued_frac": issued / FP32_MFMA_PEAK,
                    "issued_rows_per_launch": r["rows_per_launch"]})
        if kernel.startswith("rollout_v2_kernel<64, true"):
            out["note"] = ("fp32 algorithmic FLOPs vs the fp32 MFMA peak; the GRU products run as split-bf16 fp32 "
                           "emulation (6 bf16 MFMA partial products each, DESIGN.md §4a)")
    return out


def cpu_baselines(legs, a):
    """The CPU legs on the host cores, in a child process that never touches the GPU (it also forks the
    process-model leg's env workers): oracle/cpu_baseline.py. ``legs``: "vector", "process", "refil"."""
    cmd = [sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--json", "--seconds",
           str(a.cpu_seconds), "--episode-limit", str(a.episode_limit), "--legs", ",".join(legs)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=max(300, 8 * len(legs) * a.cpu_seconds))
    if p.returncode != 0:
        return {"error": p.stderr[-400:]}
    return json.loads(p.stdout.strip().splitlines()[-1])


def cpu_entry(c, leg_names):
    """The cpu_baseline object of one bench leg from the CPU run's legs (the first named leg is ``value``)."""
    if "error" in c:
        return {"value": None, "unit": "env-steps/s", "error": c["error"]}
    legs = [x for x in c["legs"] if x["leg"] in leg_names]
    main_leg = legs[0]
    return {"value": main_leg["value"], "unit": "env-steps/s", "cores": main_leg["cores"], "kind": "port",
            "sample": main_leg["sample"], "cpu_model": c.get("cpu_model"), "host_cpus": c.get("host_cpus"),
            "per_gpu_core_share": c.get("per_gpu_core_share"), "usable_cpus": c.get("usable_cpus"),
            "legs": legs}


# ---- N > 1 without an outer launcher: start the ranks ourselves -----------------------------------------------
def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a, argv, out_fd) -> int:
    """``bench.py --gpus N`` (N > 1) run directly, without torch.distributed.run around it: start
    ``python -m torch.distributed.run --nproc-per-node N bench.py <same args>`` as a CHILD process (this process has
    made no GPU call -- only ``import torch`` -- so nothing is exec'd from a GPU-initialised process), one rank per
    GPU over RCCL, and relay rank 0's single JSON line. Any rank failing fails the bench (non-zero exit).
    Replaces the reference's league topology launch, src/league/processes/central_worker.py:84-97."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver (RCCL peer buffers)
    env.setdefault("OMP_NUM_THREADS", "1")
    # a rank hung in RCCL init or a collective must not hang the bench: bound the child by the run's own size
    limit = 600 + 3 * (a.steps + a.warmup) + 8 * 3 * a.cpu_seconds
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env, start_new_session=True)
    try:
        stdout, _ = proc.communicate(timeout=limit)
    except subprocess.TimeoutExpired:
        os.killpg(proc.pid, 9)  # the launcher's own process group: it and its ranks
        proc.communicate()
        sys.stderr.write(f"bench: {a.gpus}-rank launch exceeded {limit:.0f} s, killed\n")
        return 124
    p = subprocess.CompletedProcess(cmd, proc.returncode, stdout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or len(lines) != 1:
        sys.stderr.write(f"bench: {a.gpus}-rank launch failed (exit {p.returncode}, {len(lines)} result lines)\n"
                         + p.stdout[-2000:] + "\n")
        return p.returncode or 1
    os.write(out_fd, (lines[0] + "\n").encode())
    return 0


def leg_summary(L, a):
    """A non-head leg's object in the JSON line."""
    out = {"value": L["value"], "unit": "env-steps/s", "ms_per_step": L["ms_per_step"],
           "represents": L["represents"], "workload": L["workload"], "parallelism": L["parallelism"],
           "per_rank_value": L["per_rank"], "env_steps": L["env_steps"], "mean_episode_len": L["mean_episode_len"],
           "rollout_kernel": L["roofline"]["kernel"], "avg_kernel_ms": L["avg_kernel_ms"],
           "roofline_frac": L["roofline"]["frac"], "roofline": L["roofline"]}
    if "league_iterations" in L:
        out.update({"match_len": a.match_len, "league_warmup_iterations": L.get("league_warmup_iterations"),
                    **{k: L[k] for k in ("league_iterations", "exchange_ms_mean", "exchange_ms_max", "exchange_frac",
                                         "collective_backend", "world_size", "opponents_rank0",
                                         "historical_snapshots", "snapshots_taken", "historical_matches_rank0",
                                         "historical_matches_timed_rank0", "evictions", "payoff_games", "teams",
                                         "away_teams_rank0")},
                    "note": "league scaling = league.value at N / league.value at N = 1 (same leg, same per-GPU "
                            "workload: weak scaling)"})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default 1, or WORLD_SIZE under an outer torch.distributed.run")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="auto", choices=["auto", "ai", "league", "refil"])
    ap.add_argument("--match-len", type=int, default=5, help="league: training iterations per league iteration")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo for rehearsals)")
    ap.add_argument("--device", type=int, default=None, help="GPU index for every rank (rehearsal on one GPU)")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--episode-limit", type=int, default=100)
    ap.add_argument("--plan", default=None, help="match_build_plan (default medium_1h_4t; refil: refil_8)")
    ap.add_argument("--league-teams", dest="league_teams", default="composed", choices=["composed", "mirror"],
                    help="league leg: per-player TeamComposer compositions (default) or the plan mirrored")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timing-every", type=int, default=1,
                    help="HIP events around every k-th rollout launch of the timed region (0: none, A/B only; "
                         "every launch when --steps < 2k)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch / process-group plumbing only: init the group, report the world, run no leg")
    argv = sys.argv[1:]
    a = ap.parse_args(argv)
    global TIMING_EVERY
    TIMING_EVERY = a.timing_every
    # stdout carries exactly one line, the JSON result: native libraries (RCCL prints a version banner on its first
    # communicator) write to fd 1, so fd 1 is pointed at stderr and the result goes to a saved copy of stdout
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)

    launched = "WORLD_SIZE" in os.environ  # torch.distributed.run (any nproc) -> a process group, RCCL
    if a.gpus is None:  # a plain `torchrun --nproc-per-node N bench.py` takes N from the launcher
        a.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and not launched:
        sys.exit(launch_ranks(a, argv, out_fd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench: --gpus {a.gpus} but the launcher started {world} ranks")
    local_rank = a.device if a.device is not None else int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    use_gpu = not a.dry_run
    if launched:
        import torch.distributed as dist
        if use_gpu:
            torch.cuda.set_device(local_rank)
        if a.backend == "nccl" and use_gpu:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
        else:
            dist.init_process_group(a.backend)
        assert dist.get_world_size() == a.gpus, (dist.get_world_size(), a.gpus)
    dev = torch.device(f"cuda:{local_rank}") if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    ctx = Ctx(dist, dev)

    if a.dry_run:
        # the league exchange's collectives once over the launched group (payoff all_reduce, parameter all_gather,
        # barrier), with a parameter vector = the rank id, so the line shows every rank took part
        from maleague.league import DistributedLeague
        from maleague.league.payoff import PayoffEntry
        lg = DistributedLeague(n_players=world, device=dev, seed=0, max_historical=world)
        lg.record(rank, (rank + 1) % world, PayoffEntry.WIN, n=rank + 1)
        lg.sync_payoff()
        lg.exchange(torch.full((8,), float(rank), device=dev), 100 * rank, checkpoint=True)
        lg.barrier()
        ranks = ctx.gather(float(rank))
        if rank == 0:
            out = {"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": ctx.world, "steps": 0,
                   "warmup": 0, "dry_run": True, "ranks": [int(r) for r in ranks],
                   "league": {"world_size": ctx.world, "collective_backend": lg.backend,
                              "params_of": [float(lg.params_of(p)[0]) for p in range(world)],
                              "payoff_wins": float(lg.payoff.tensor[..., PayoffEntry.WIN].sum()),
                              "historical_snapshots": len(lg.historical_meta)}}
            os.write(out_fd, (json.dumps(out) + "\n").encode())
        if dist:
            dist.destroy_process_group()
        return

    from maleague.custom_logging import MainLogger
    from maleague.runs import MultiAgentExperiment

    legs = {"auto": ["ai", "league", "refil"], "ai": ["ai"], "league": ["league"], "refil": ["refil"]}[a.mode]
    results = {}
    for leg in legs:
        args, plan = make_args(leg, a, rank, local_rank)
        inst = None
        if leg in ("ai", "refil"):
            exp = MultiAgentExperiment(args, MainLogger(log_interval=10 ** 12))
            exp._init_stepper()
            if leg == "refil":
                ea = args.env_args
                workload = (f"refil_{plan}_{ea.get('min_agents', 3)}to{ea.get('max_agents', 8)}agents_{a.envs}envs_"
                            f"ep{a.episode_limit}")
                cfg_name = "BASELINE config 5 (REFIL, 3-8 agents per env, 4096 envs per GPU)"
            else:
                workload = f"qmix_5v5_{plan}_{a.envs}envs_ep{a.episode_limit}"
                cfg_name = "BASELINE config 2 (QMIX 5v5, 4096 envs per GPU, one learner per GPU vs scripted AI)"
            parallelism = f"replicas{world}"
        else:
            from maleague.league import DistributedLeague, LeagueInstance
            lg = DistributedLeague(n_players=world, device=dev, seed=0, max_historical=4 * world)
            lmode, roles = league_setup(world, args)
            pteams, n_teams = league_teams(world, a)
            inst = LeagueInstance(args, MainLogger(log_interval=10 ** 12), lg, mode=lmode, role=roles, seed=0,
                                  teams=pteams)
            workload, cfg_name = league_workload(world, plan, a, roles, n_teams)
            exp = inst.experiment
            parallelism = f"league{world}_{lg.backend}"
        stepper = exp.stepper
        B = stepper.batch_size
        stepper.t_env = 10 ** 6  # steady-state exploration (epsilon floor 0.05), SURVEY §8d
        if inst is None:
            ep = [0]

            def iteration(i, exp=exp, ep=ep):
                # one iteration of MultiAgentExperiment.start's loop (train-mode run, insert, train, the
                # interval checks), exactly as the product loop runs it
                ep[0] = exp._iteration(ep[0])

            r = timed_loop(ctx, iteration, stepper, a.steps, a.warmup)
        else:
            r = run_league_leg(ctx, inst, a.steps, a.warmup, a.match_len)
        r["roofline"] = roofline(leg, stepper, r, a.steps, B)
        r.update({"workload": workload, "represents": cfg_name, "parallelism": parallelism, "envs_per_gpu": B,
                  "mean_episode_len": r["env_steps"] / max(1, a.steps * B * world)})
        results[leg] = r
        del exp, inst, stepper
        torch.cuda.empty_cache()

    head = legs[0]
    h = results[head]
    cpu, cpu_refil = None, None
    if rank == 0 and world == 1 and head in ("ai", "refil") and not a.no_cpu_baseline:
        names = (["vector", "process"] if head == "ai" else []) + (["refil"] if "refil" in results else [])
        c = cpu_baselines(names, a)
        cpu = cpu_entry(c, ["refil"] if head == "refil" else ["vector", "process"])
        if head != "refil" and "refil" in results:
            cpu_refil = cpu_entry(c, ["refil"])
    if rank == 0:
        out = {"metric": METRIC, "value": h["value"], "unit": "env-steps/s", "n_gpus": world, "steps": a.steps,
               "warmup": a.warmup, "ms_per_step": h["ms_per_step"], "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "f32",
               "data": ("synthetic (entity battles, 3-8 agents per env padded to 8, random-init REFIL)"
                        if head == "refil" else "synthetic (spec-v1 5v5 battles, random-init QMIX)"),
               "config": {"workload": h["workload"], "represents": h["represents"], "mode": a.mode,
                          "envs_per_gpu": h["envs_per_gpu"], "episode_limit": a.episode_limit, "learner_batch": 32,
                          "rnn_hidden_dim": 64, "buffer_size": 5000, "parallelism": h["parallelism"],
                          **({"match_len": a.match_len} if head == "league" else {})},
               "env_steps": h["env_steps"], "mean_episode_len": h["mean_episode_len"],
               "per_rank_value": h["per_rank"], "roofline": h["roofline"], "cpu_baseline": cpu}
        if head == "league":
            out["league"] = {k: h[k] for k in ("league_iterations", "exchange_ms_mean", "exchange_ms_max",
                                               "exchange_frac", "collective_backend", "world_size",
                                               "opponents_rank0", "historical_snapshots", "snapshots_taken",
                                               "historical_matches_rank0", "historical_matches_timed_rank0",
                                               "evictions", "teams", "away_teams_rank0")}
        if "league" in results and head != "league":
            out["league"] = leg_summary(results["league"], a)
        if "refil" in results and head != "refil":
            out["refil"] = leg_summary(results["refil"], a)
            out["refil"]["cpu_baseline"] = cpu_refil
            out["refil"]["note"] = ("BASELINE config 5 at the same N (replicas: one REFIL learner per GPU vs the "
                                    "scripted AI)")
        sys.stdout.flush()
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
