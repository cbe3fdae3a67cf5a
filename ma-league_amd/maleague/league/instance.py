"""One league player per rank: the training loop of a league instance.

Restates the per-process loop of src/league/processes/training/matchmaking_league_instance.py:19-71 and
role_based_league_instance.py:21-53 (with LeagueExperimentInstance, league_experiment_process.py:57-105):
  1. (optional) pre-train the home policy against the mirrored scripted AI     (:21-25)
  2. share the home agent's parameters with the league                          (:26)
  3. per league iteration: get a match (matchmaker or league role), load the adversary's parameters, play
     ``iterations_per_match`` self-play training iterations recording every episode's result, share.
Processes, queues and the coordinator are replaced by one rank per GPU and DistributedLeague collectives.
The self-play experiment is built once per instance and its adversary swapped between matches (the
reference rebuilds LeagueExperiment -- replay buffer, optimizer state -- for every match).
"""
from __future__ import annotations

import copy

import numpy as np
import torch
import torch.distributed as dist

from ..envs.plans import mirror_plan
from ..runs import LeagueExperiment, MultiAgentExperiment
from ..runs.sp_ma_experiment import agent_vector, load_agent_vector
from .distributed import DistributedLeague
from .matchmaking import REGISTRY as matchmaking_REGISTRY
from .roles import ROLES, Historical, LeagueView, alphastar_roles
from .teams import match_plan


class LeagueInstance:
    """``mode``: "matchmaking" (args.matchmaking in pfsp/uniform/random/fsp/adversaries, every player a
    learner) or "rolebased" (``role`` in simple/main/main_exploiter/league_exploiter)."""

    def __init__(self, args, logger, league: DistributedLeague, mode="matchmaking", role=None, seed=0,
                 experiment=None, teams=None):
        """``teams``: the league's Team of every player (index = pid; league.teams.compose_league_teams, one team
        per player as CentralWorker assigns them, central_worker.py:84-93). Each match then puts this player's team
        against the opponent's (a historical snapshot plays its parent's team). None: every player plays the
        env config's own plan, mirrored."""
        self.args, self.logger, self.league = args, logger, league
        self.pid = league.player()
        self.mode = mode
        if teams is not None and len(teams) != league.n:
            raise ValueError(f"{len(teams)} teams for a league of {league.n} players (one team per player)")
        self.teams = list(teams) if teams is not None else None
        self.home_team = self.teams[self.pid] if self.teams is not None else None
        self.away_team = None
        self.away_teams = []  # the away roster (codes) of every match, in order
        rng = np.random.RandomState(seed * 1000 + self.pid)
        if mode == "rolebased":
            roles = role if isinstance(role, (list, tuple)) else [role or "simple"] * league.n
            kw = dict(checkpoint_min_steps=float(getattr(args, "league_checkpoint_min_steps", 2e9)),
                      checkpoint_max_steps=float(getattr(args, "league_checkpoint_max_steps", 4e9)))
            # every rank holds the full player table (roles are needed by the others' matchmaking)
            self.players = [ROLES[r](pid, np.random.RandomState(seed * 1000 + pid), **kw) for pid, r in enumerate(roles)]
            self.me = self.players[self.pid]
            self.matchmaker = None
        else:
            self.players = [ROLES["simple"](pid) for pid in range(league.n)]
            self.me = self.players[self.pid]
            self.matchmaker = matchmaking_REGISTRY[getattr(args, "matchmaking", "pfsp")](
                rng, record_match=league.record_match)
        if experiment is None:
            sp_args = copy.deepcopy(args)
            sp_args.env_args = dict(args.env_args)
            sp_args.env_args["match_build_plan"] = self._plan(ai=False)
            experiment = LeagueExperiment(sp_args, logger)
            experiment._init_stepper()
        self.experiment = experiment
        self.opponent = None
        self.history = []  # (league iteration, opponent pid, historical?)
        self.episode = 0

    def _plan(self, ai: bool):
        """The home team mirrored (league_experiment_process.py:57-62 with away=None): this player's league team,
        or the env config's own plan when the league has no team compositions."""
        if self.home_team is not None:
            return match_plan(self.home_team, ai=ai)
        return mirror_plan(self.args.env_args["match_build_plan"], ai=ai, config_dir=getattr(self.args, "config_dir", None))

    def team_of(self, pid: int):
        """The Team a league pid plays: a player's own, a historical snapshot its parent's (None without teams)."""
        if self.teams is None:
            return None
        if pid < self.league.n:
            return self.teams[pid]
        parents = [p for h, p, _ in self.league.historical_meta if h == pid]
        if not parents:
            raise KeyError(f"league pid {pid} is neither a player nor a stored historical snapshot")
        return self.teams[parents[0]]

    # ---- phases -------------------------------------------------------------------------------------------
    def pretrain_vs_ai(self, iterations: int = 0, play_time_seconds: float = None):
        """matchmaking_league_instance.py:21-25: initial play against the mirrored scripted AI, for ``iterations``
        training iterations or ``play_time_seconds`` of wall time (the reference's play_time_mins)."""
        if iterations <= 0 and not play_time_seconds:
            return
        ai_args = copy.deepcopy(self.args)
        ai_args.env_args = dict(self.args.env_args)
        ai_args.env_args["match_build_plan"] = self._plan(ai=True)
        exp = MultiAgentExperiment(ai_args, self.logger)
        load_agent_vector(exp.home_mac, agent_vector(self.experiment.home_mac))
        if play_time_seconds:
            exp.start(play_time_seconds=play_time_seconds)
        else:
            exp.start(max_iterations=iterations)
        self.experiment.load_home_agent(exp.home_mac.agent.state_dict())
        del exp

    def view(self) -> LeagueView:
        hist = [Historical(pid, parent, steps) for pid, parent, steps in self.league.historical_meta]
        # the host copy of this league iteration's payoff (DistributedLeague.host_snapshot) when there is one
        pay = self.league.payoff_host if self.league.payoff_host is not None else self.league.payoff
        return LeagueView(pay, self.players, hist)

    def sync(self):
        """League iteration boundary: payoff all_reduce, parameter / checkpoint all_gather, barrier, next match.
        Returns (opponent pid, historical?) or None when the matchmaker ends the league for this player."""
        home = self.experiment.home_mac
        self.league.sync_payoff()
        # payoff + this player's trained steps in one device -> host read (matchmaking then runs on the host copy)
        agent = home.agent
        counter = agent.trained_counter(self.league.device) if hasattr(agent, "trained_counter") else None
        dev_steps = self.league.host_snapshot(counter)
        steps = agent.trained_steps_with(dev_steps) if counter is not None else int(agent.trained_steps)
        self.me.trained_steps = steps
        ckpt = self.me.ready_to_checkpoint(self.view()) if self.mode == "rolebased" else False
        taken = self.league.exchange(agent_vector(home), steps, ckpt)
        if ckpt and any(parent == self.pid for _, parent in taken):
            self.me.checkpoint()  # only when the snapshot exists (max_historical > 0): otherwise it asks again
        self.league.barrier()
        view = self.view()
        if self.matchmaker is not None:
            opp, hist = self.matchmaker.get_match(self.pid, view), False
        else:
            opp, hist = self.me.get_match(view)
            self.league.record_match(self.pid, opp)
        # the league ends for everybody once one player has no match left (keeps the collectives aligned)
        if self._any(opp is None):
            return None
        self.opponent = int(opp)
        self.experiment.load_adversary_vector(self.league.params_of(self.opponent))
        if self.teams is not None:  # the adversary's roster (matchmaking_league_instance.py:52, :61-62)
            self.away_team = self.team_of(self.opponent)
            self.away_teams.append(self.away_team.codes())
            self.experiment.configure_match(self.home_team, self.away_team)
        self.history.append((len(self.history), self.opponent, bool(hist)))
        return self.opponent, hist

    def _any(self, flag: bool) -> bool:
        if not self.league._dist:
            return bool(flag)
        t = torch.tensor([1.0 if flag else 0.0],
                         device="cpu" if dist.get_backend() == "gloo" else self.league.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return bool(t.item() > 0)

    def play(self, iterations: int):
        """Self-play training iterations against the current opponent, every episode's result recorded into
        the local payoff delta on the device (league_experiment_process.py:96-105 via on_episode_end)."""
        exp, st = self.experiment, self.experiment.stepper
        B = st.batch_size
        for _ in range(iterations):
            exp._train_episode(self.episode)
            info = st.last_run_info() if hasattr(st, "last_run_info") else st._info
            self.league.record_runs(self.pid, self.opponent, info[B:3 * B].view(B, 2), info[3 * B:4 * B])
            self.episode += B

    def play_for(self, seconds: float, max_iterations: int = None) -> int:
        """A match of ``seconds`` wall time (the reference's ``start(play_time_seconds=play_time_mins * 60)``,
        matchmaking_league_instance.py:64): training iterations until the time is up (at least one), or
        ``max_iterations``. Returns the iterations played. Ranks play their matches independently; they meet
        again at the next sync()."""
        import time
        t0, n = time.perf_counter(), 0
        while n == 0 or (time.perf_counter() - t0 < seconds and (max_iterations is None or n < max_iterations)):
            self.play(1)
            n += 1
        return n

    def run(self, league_iterations: int, iterations_per_match: int, pretrain_iterations: int = 0):
        self.pretrain_vs_ai(pretrain_iterations)
        for _ in range(league_iterations):
            if self.sync() is None:
                break
            self.play(iterations_per_match)
        self.league.sync_payoff()
        return self.history


def league_roles_for(world: int, args) -> list:
    """Config 3 (2 learners): PFSP self-play between simple players; config 4 (>= 4 ranks): AlphaStar roles
    (half main players, half main exploiters unless league_main_agents / league_main_exploiters say otherwise)."""
    if world < 4:
        return ["simple"] * world
    return alphastar_roles(world, getattr(args, "league_main_agents", None),
                           getattr(args, "league_main_exploiters", None),
                           int(getattr(args, "league_league_exploiters", 0)))
