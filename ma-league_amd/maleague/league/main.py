"""League entry point: ``src/central_worker_main.py:28-111`` + ``CentralWorker.run`` (``central_worker.py:33-121``),
one rank per GPU.

The reference starts a CentralWorker process that composes the league's teams, then one training process per
team, an agent-pool process and a shared-memory payoff tensor. Here every rank of a ``torch.distributed``
launch is one league player on its own GPU; the exchange runs over RCCL (``DistributedLeague``)::

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        ma-league_amd/maleague/league/main.py --config=qmix --env-config=ma --league-config=matchmaking \\
        --experiment=alphastar --league_size=4 --team_size=5 --runner=parallel --batch_size_run=4096 \\
        force-unit --role=HEALER --attack=RANGED

Arguments (``central_worker_main.py:37-76``): ``--team_size``, ``--league_size``, ``--experiment``
(``matchmaking``: one learner per team, opponents by ``--matchmaking``; ``rolebased``: SimpleLeague, one
SimplePlayer per team (``simple_league.py:26-47``); ``alphastar``: AlphaStarLeague made functional -- per team one
main player, ``--main_exploiters_n`` main exploiters and ``--league_exploiters_n`` league exploiters
(``alpha_star_league.py:23-40``); the reference's ``ensemble`` experiment is out of scope),
``--matchmaking``, ``--balance-cuda-workload``, ``--league-config``, ``--env-config``, ``--config``, and the
``force-unit --role --attack [--unique]`` subcommand. Every other ``--key=value`` overrides the layered YAML
config (the reference's nestargs over-parse, ``config_builder.py:51-55``; string values included).
``--config-dir`` reads the reference's own ``src/config`` tree; without it the built-in layers are used.

Time: each match and the pre-training against the mirrored AI last ``play_time_mins`` of wall time, the league
``league_runtime_hours`` (``leagues/matchmaking.yaml:1-2``, ``matchmaking_league_instance.py:25,32-36,64``). The
stop decision is rank 0's, broadcast before every league iteration, so the collectives of all ranks stay aligned.
``--league-iterations`` / ``--match-iterations`` / ``--pretrain-iterations`` bound those phases by iteration counts
instead (tests, benchmarks).

Output: rank 0 writes ``<local_results_path>/league_<token>/league_config.json`` (arguments + every player's team,
role and device) and ``payoff.json`` and prints the payoff per team like ``CentralWorker._print_payoff``
(``central_worker.py:123-131``); the last stdout line is a JSON summary.
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time

if __package__ in (None, ""):  # run as a script (torch.distributed.run <path>/main.py)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from maleague.league.matchmaking import REGISTRY as MATCHMAKING_REGISTRY  # noqa: E402
from maleague.league.teams import RoleTypes, UnitAttackTypes, compose_league_teams  # noqa: E402

EXPERIMENTS = ("matchmaking", "rolebased", "alphastar")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="maleague.league.main", description=__doc__.split("\n\n")[0])
    sub = p.add_subparsers(dest="cmd", help="Sub-Commands")
    p.add_argument("--team_size", default=5, type=int, help="Define how many agents comprise a team.")
    p.add_argument("--league_size", default=2, type=int, help="Define the size of the league (= how many teams)")
    p.add_argument("--experiment", default=EXPERIMENTS[0], choices=EXPERIMENTS,
                   help="Define the type of experiment to run.")
    p.add_argument("--matchmaking", default=None, choices=sorted(MATCHMAKING_REGISTRY),
                   help="Matchmaking of the matchmaking experiment (default: the league config's, else pfsp).")
    p.add_argument("--balance-cuda-workload", dest="balance_cuda_workload", action="store_true",
                   help="Round-robin players over the visible GPUs (default: rank r on LOCAL_RANK's GPU).")
    p.add_argument("--league-config", dest="league_config", required=True, help="Define which league to use.")
    p.add_argument("--env-config", dest="env_config", required=True, help="Define which env to use.")
    p.add_argument("--config", required=True, help="Define which algorithm to use.")
    p.add_argument("--config-dir", dest="config_dir", default=None,
                   help="A config tree (the reference's src/config); default: the built-in layers.")
    # AlphaStar roles per team (alpha_star_league.py:8-21)
    p.add_argument("--main_exploiters_n", type=int, default=1)
    p.add_argument("--league_exploiters_n", type=int, default=0)
    # launch / run bounds (extensions)
    p.add_argument("--backend", default=None, help="torch.distributed backend (default nccl = RCCL on GPUs, else gloo)")
    p.add_argument("--device", type=int, default=None, help="GPU index for every rank (rehearsals on one GPU)")
    p.add_argument("--league-iterations", dest="league_iterations", type=int, default=None)
    p.add_argument("--match-iterations", dest="match_iterations", type=int, default=None)
    p.add_argument("--pretrain-iterations", dest="pretrain_iterations", type=int, default=None)
    p.add_argument("--max-historical", dest="max_historical", type=int, default=None,
                   help="historical snapshot slots (default 4 per player)")
    p.add_argument("--seed", type=int, default=None, help="league seed (teams, matchmaking); default: config seed or 0")
    p.add_argument("--dry-run", dest="dry_run", action="store_true",
                   help="compose teams, assign players, run one league exchange; no training")
    f = sub.add_parser("force-unit", help="Forces the team composer to create teams with one or more specified "
                                          "unit(s). A unit is specified via its role and attack type.")
    f.add_argument("--role", choices=[m.name for m in RoleTypes], type=str.upper, default=list(RoleTypes)[0].name,
                   help="Define a role of an unit the team has to contain")
    f.add_argument("--attack", choices=[m.name for m in UnitAttackTypes], type=str.upper,
                   default=list(UnitAttackTypes)[0].name, help="Define an attack type of an unit the team has to contain")
    f.add_argument("--unique", dest="unique", action="store_true",
                   help="Enforce the desired unit within a team to be unique.")
    f.set_defaults(unique=True)
    return p


def parse(argv):
    """(league arguments, config overrides): unknown ``--key=value`` tokens become config overrides."""
    a, extra = build_parser().parse_known_args(argv)
    overrides = []
    for tok in extra:
        if not tok.startswith("--") or "=" not in tok:
            raise SystemExit(f"league: cannot parse argument {tok!r} (config overrides look like --key=value)")
        overrides.append(tok)
    if a.cmd != "force-unit":
        a.role = a.attack = None
        a.unique = False
    return a, overrides


def player_layout(experiment: str, league_size: int, main_exploiters_n: int = 1, league_exploiters_n: int = 0):
    """(roles, team index) of every player. matchmaking / rolebased: one player per team (central_worker.py:84-93,
    simple_league.py:29-45); alphastar: per team a main player, then its exploiters (alpha_star_league.py:23-40)."""
    if experiment == "matchmaking":
        return [None] * league_size, list(range(league_size))
    if experiment == "rolebased":
        return ["simple"] * league_size, list(range(league_size))
    if experiment == "alphastar":
        per_team = ["main"] + ["main_exploiter"] * main_exploiters_n + ["league_exploiter"] * league_exploiters_n
        roles, team_idx = [], []
        for t in range(league_size):
            roles += per_team
            team_idx += [t] * len(per_team)
        return roles, team_idx
    raise NotImplementedError(f"Experiment not supported: {experiment}")


class _Stop:
    """Rank 0's stop decision, broadcast (league_runtime_hours / --league-iterations)."""

    def __init__(self, dist, dev):
        self.dist, self.dev = dist, dev

    def __call__(self, stop: bool) -> bool:
        if self.dist is None:
            return stop
        import torch
        t = torch.tensor([1 if stop else 0], dtype=torch.int32, device=self.dev)
        self.dist.broadcast(t, src=0)
        return bool(t.item())


def _print_payoff(payoff, teams, player_team, roles):
    """CentralWorker._print_payoff (central_worker.py:123-131), per player (the same team may field several)."""
    from maleague.league.payoff import PayoffEntry
    n = len(player_team)
    for pid in range(n):
        team = teams[player_team[pid]]
        role = f" as {roles[pid]}" if roles[pid] else ""
        print(f"Stats for {team} ({team.codes()}) from instance {pid}{role}")
        for entry in PayoffEntry:
            print(f"{entry.name.capitalize()} {payoff[pid, :n, entry].tolist()}")


def main(argv=None) -> dict:
    import torch
    a, overrides = parse(sys.argv[1:] if argv is None else argv)
    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    roles, team_idx = player_layout(a.experiment, a.league_size, a.main_exploiters_n, a.league_exploiters_n)
    if len(roles) != world:
        raise SystemExit(f"league: the {a.experiment} experiment with league_size={a.league_size} has {len(roles)} "
                         f"players, the launch has {world} ranks (one league player per rank / GPU)")
    use_gpu = torch.cuda.is_available() and not a.dry_run
    if use_gpu:
        n_dev = torch.cuda.device_count()
        dev_idx = a.device if a.device is not None else (rank % n_dev if a.balance_cuda_workload else local_rank)
        torch.cuda.set_device(dev_idx)
        dev = torch.device(f"cuda:{dev_idx}")
    else:
        dev_idx, dev = 0, torch.device("cpu")
    dist = None
    if launched:
        import torch.distributed as dist
        backend = a.backend or ("nccl" if use_gpu else "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    cdev = dev if (dist is not None and dist.get_backend() == "nccl") else torch.device("cpu")

    from maleague.utils.config import build_config, to_args
    cfg = build_config(a.config, a.env_config, league=a.league_config, overrides=overrides, config_dir=a.config_dir,
                       device_index=dev_idx, cuda_available=use_gpu)
    seed = a.seed if a.seed is not None else int(cfg.get("seed", 0) or 0)
    matchmaking = a.matchmaking or cfg.get("matchmaking", "pfsp")
    # teams: composed identically on every rank (seeded), rank 0's composition broadcast as the one in force
    teams = compose_league_teams(a.team_size, a.league_size, a.role, a.attack, a.unique, seed=seed)
    if dist is not None:
        tids = [[t.tid for t in teams]]
        dist.broadcast_object_list(tids, src=0)
        if tids[0] != [t.tid for t in teams]:
            raise RuntimeError(f"league: rank {rank} composed teams {[t.tid for t in teams]}, rank 0 {tids[0]}")
    player_teams = [teams[i] for i in team_idx]
    cfg["seed"] = seed + rank  # per-instance seed (experiment_process.py:102-107)
    cfg["matchmaking"] = matchmaking
    args = to_args(cfg)

    from maleague.league import DistributedLeague, LeagueInstance, PayoffEntry
    max_hist = a.max_historical if a.max_historical is not None else 4 * world
    lg = DistributedLeague(n_players=world, device=dev, seed=seed, max_historical=max_hist)
    token = datetime.datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    log_dir = os.path.join(cfg.get("local_results_path", "results"), f"league_{token}")
    layout = [{"pid": p, "role": roles[p], "team": player_teams[p].to_json(), "codes": player_teams[p].codes()}
              for p in range(world)]
    summary = {"world_size": world, "experiment": a.experiment, "matchmaking": matchmaking, "seed": seed,
               "force_unit": [a.role, a.attack, a.unique] if a.role else None, "team_tids": [t.tid for t in teams],
               "players": layout, "collective_backend": lg.backend}

    if a.dry_run:
        # plumbing only: one league exchange (payoff all_reduce, parameter all_gather, barrier) with a parameter
        # vector that names its player's team, so the summary shows every rank took part with its own roster
        lg.record(rank, (rank + 1) % world, PayoffEntry.WIN, n=rank + 1)
        lg.sync_payoff()
        lg.exchange(torch.full((4,), float(player_teams[rank].tid), device=dev), 0, checkpoint=False)
        lg.barrier()
        summary["params_of"] = [float(lg.params_of(p)[0]) for p in range(world)]
        summary["payoff_wins"] = float(lg.payoff.tensor[..., 1].sum())
    else:
        from maleague.custom_logging import MainLogger
        logger = MainLogger(args=args)
        inst = LeagueInstance(args, logger, lg, mode="matchmaking" if roles[0] is None else "rolebased",
                              role=None if roles[0] is None else roles, seed=seed, teams=player_teams)
        play_s = float(cfg.get("play_time_mins", 1.0)) * 60.0
        runtime_s = float(cfg.get("league_runtime_hours", 0.0)) * 3600.0
        if a.pretrain_iterations is not None:
            inst.pretrain_vs_ai(iterations=a.pretrain_iterations)
        else:
            inst.pretrain_vs_ai(play_time_seconds=play_s)
        stop = _Stop(dist, cdev)
        t0, iters, matches = time.time(), 0, []
        while True:
            over = (a.league_iterations is not None and iters >= a.league_iterations) or \
                   (a.league_iterations is None and time.time() - t0 > runtime_s)
            if stop(over):
                break
            if inst.sync() is None:  # no match left for some player: the league ends for everybody
                break
            n = inst.play_for(play_s if a.match_iterations is None else float("inf"), a.match_iterations)
            matches.append({"opponent": inst.opponent, "historical": bool(inst.history[-1][2]), "iterations": n,
                            "away_team": inst.away_team.tid if inst.away_team is not None else None,
                            "away_codes": inst.away_team.codes() if inst.away_team is not None else None})
            iters += 1
        lg.sync_payoff()
        if use_gpu:
            torch.cuda.synchronize(dev)
        summary.update({"league_iterations": iters, "t_env": int(inst.experiment.stepper.t_env),
                        "historical_snapshots": len(lg.historical_meta)})
        gathered = [None] * world
        if dist is not None:
            dist.all_gather_object(gathered, matches)
        else:
            gathered = [matches]
        summary["matches"] = gathered
        summary["payoff"] = lg.payoff.tensor.cpu().tolist()
    if rank == 0:
        os.makedirs(log_dir, exist_ok=True)
        with open(os.path.join(log_dir, "league_config.json"), "w") as f:
            json.dump({"args": {k: v for k, v in vars(a).items()}, "overrides": overrides, **summary}, f, indent=2,
                      default=str)
        if "payoff" in summary:
            with open(os.path.join(log_dir, "payoff.json"), "w") as f:
                json.dump(summary["payoff"], f)
            import torch as _t
            _print_payoff(_t.tensor(summary["payoff"]), teams, team_idx, roles)
        summary["log_dir"] = log_dir
        print(json.dumps(summary, default=str), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return summary


if __name__ == "__main__":
    main()
