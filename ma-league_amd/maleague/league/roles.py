"""League roles: the AlphaStar players and the simple PFSP player, made functional.

Restates src/league/rolebased/alphastar/main_player.py:11-132, exploiters.py:8-118, players.py:11-66,
simple/simple_player.py:14-47 and utils/helpers.py:4-12. In the reference these classes are scaffolding
(constructor signatures that do not match their callers, HistoricalPlayer calling object.__init__ with an
argument, checkpoints raising NotImplementedError). Here every player is an index into
one replicated league state (``LeagueView``): pids 0..R-1 are the learning players (one per rank),
pids >= R are historical snapshots (checkpoints) with a parent pid. ``get_match`` returns
``(opponent_pid, is_historical)``; matchmaking never touches parameters (those live in the AgentPool).

Decisions where the reference has no working behaviour (listed in DESIGN.md):
* a branch that finds no candidate (no historical players yet) falls back to the main-player self-play
  branch instead of ending the league (main_player.py:57-58, exploiters.py:89-90 return None);
* checkpoint thresholds (2e9 / 4e9 trained steps, main_player.py:121-132) are configurable.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

from .payoff import PayoffEntry, PFSPSampling


def remove_monotonic_suffix(win_rates, players):
    """utils/helpers.py:4-12: drop the trailing run of checkpoints whose win rate only increases."""
    if win_rates is None or len(win_rates) == 0:
        return win_rates, players
    for i in range(len(win_rates) - 1, 0, -1):
        if win_rates[i - 1] < win_rates[i]:
            return win_rates[:i + 1], players[:i + 1]
    return np.array([]), []


@dataclass
class Historical:
    pid: int
    parent: int
    trained_steps: int = 0


@dataclass
class LeagueView:
    """What matchmaking reads: the replicated payoff (win rates) and the player table."""
    payoff: object  # PayoffWrapper
    players: list   # pid -> Player (learning players, 0..R-1)
    historical: List[Historical] = field(default_factory=list)

    def win_rates(self, pid, opponents) -> np.ndarray:
        if len(opponents) == 0:
            return np.zeros(0)
        t = self.payoff.tensor
        if t.device.type == "cpu":  # the league iteration's host copy: the same float32 arithmetic in numpy
            row = t.detach().numpy()[pid, list(opponents)]
            games = row[:, PayoffEntry.GAMES]
            with np.errstate(divide="ignore", invalid="ignore"):
                wr = (row[:, PayoffEntry.WIN] + np.float32(0.5) * row[:, PayoffEntry.DRAW]) / games
            wr[games == 0.0] = 0.5
            return wr
        return self.payoff.win_rates(pid, list(opponents)).detach().cpu().numpy()

    def of_type(self, cls) -> list:
        return [p for p in self.players if isinstance(p, cls)]

    def historical_of(self, parents=None) -> List[int]:
        return [h.pid for h in self.historical if parents is None or h.parent in parents]


class Player:
    """players.py:11-40. trained_steps mirrors the agent's (BasicMAC.update_trained_steps)."""

    def __init__(self, pid: int, rng: Optional[np.random.RandomState] = None, checkpoint_min_steps: float = 2e9,
                 checkpoint_max_steps: float = 4e9):
        self.pid = pid
        self.rng = rng or np.random.RandomState(pid)
        self.trained_steps = 0
        self._checkpoint_step = 0
        self._pfsp = PFSPSampling(self.rng)
        self.min_steps, self.max_steps = checkpoint_min_steps, checkpoint_max_steps

    def get_match(self, league: LeagueView) -> Tuple[int, bool]:
        raise NotImplementedError()

    def is_main_player(self) -> bool:
        return False

    def ready_to_checkpoint(self, league: LeagueView) -> bool:
        return False

    def checkpoint(self):
        self._checkpoint_step = self.trained_steps

    def _pfsp_pick(self, league, cands, weighting) -> int:
        return int(self._pfsp.sample(cands, prio_measure=league.win_rates(self.pid, cands), weighting=weighting))

    def __str__(self):
        return f"{type(self).__name__}_{self.pid}"


class SimplePlayer(Player):
    """simple_player.py:14-47: PFSP ("squared") over every current agent of the pool (self included)."""

    def is_main_player(self):
        return True

    def get_match(self, league):
        opponents = [p.pid for p in league.players]
        return self._pfsp_pick(league, opponents, "squared"), False

    def ready_to_checkpoint(self, league):
        return self.trained_steps - self._checkpoint_step >= self.min_steps


class MainPlayer(Player):
    """main_player.py:11-132."""

    def is_main_player(self):
        return True

    def get_match(self, league):
        coin = self.rng.random_sample()
        if coin < 0.5:  # make sure the league can be beaten: PFSP against historical players (:33-35)
            hist = league.historical_of()
            if hist:
                return self._pfsp_pick(league, hist, "squared"), True
        mains = league.of_type(MainPlayer)
        opponent = mains[self.rng.randint(len(mains))]
        if coin < 0.5 + 0.15:  # verify that no rare player was omitted (:42-46)
            req = self._verification_branch(league, opponent)
            if req is not None:
                return req
        return self._selfplay_branch(league, opponent)

    def _selfplay_branch(self, league, opponent):
        """:64-86: SP against a main player unless it is too strong -> its checkpoints (PFSP 'variance')."""
        if league.win_rates(self.pid, [opponent.pid])[0] > 0.3:
            return opponent.pid, False
        hist = league.historical_of([opponent.pid])
        if not hist:
            return opponent.pid, False
        return self._pfsp_pick(league, hist, "variance"), True

    def _verification_branch(self, league, opponent):
        """:88-118: exploited by an exploiter checkpoint (< 0.3) or forgetting a main-player checkpoint (< 0.7)."""
        exploiters = {p.pid for p in league.of_type(MainExploiter)}
        exp_hist = league.historical_of(exploiters)
        wr = league.win_rates(self.pid, exp_hist)
        if len(wr) and wr.min() < 0.3:
            return self._pfsp_pick(league, exp_hist, "squared"), True
        hist = league.historical_of([opponent.pid])
        wr = league.win_rates(self.pid, hist)
        wr, hist = remove_monotonic_suffix(wr, hist)
        if len(wr) and wr.min() < 0.7:
            return self._pfsp_pick(league, list(hist), "squared"), True
        return None

    def ready_to_checkpoint(self, league):
        """:120-132."""
        steps = self.trained_steps - self._checkpoint_step
        if steps < self.min_steps:
            return False
        hist = league.historical_of()
        wr = league.win_rates(self.pid, hist)
        return (len(wr) > 0 and wr.min() > 0.7) or steps > self.max_steps


class MainExploiter(Player):
    """exploiters.py:8-64: exploits the main players (PFSP 'variance' over their checkpoints when too strong)."""

    def get_match(self, league):
        mains = league.of_type(MainPlayer)
        opponent = mains[self.rng.randint(len(mains))]
        if league.win_rates(self.pid, [opponent.pid])[0] > 0.1:
            return opponent.pid, False
        hist = league.historical_of([opponent.pid])
        if not hist:
            return opponent.pid, False
        return self._pfsp_pick(league, hist, "variance"), True

    def ready_to_checkpoint(self, league):
        steps = self.trained_steps - self._checkpoint_step
        if steps < self.min_steps:
            return False
        mains = [p.pid for p in league.of_type(MainPlayer)]
        wr = league.win_rates(self.pid, mains)
        return (len(wr) > 0 and wr.min() > 0.7) or steps > self.max_steps


class LeagueExploiter(Player):
    """exploiters.py:67-118: PFSP ('linear_capped') over every checkpoint of the league."""

    def get_match(self, league):
        hist = league.historical_of()
        if not hist:  # reference: (None, None) -> the instance ends; here: play a main player
            mains = league.of_type(MainPlayer) or league.players
            return mains[self.rng.randint(len(mains))].pid, False
        return self._pfsp_pick(league, hist, "linear_capped"), True

    def ready_to_checkpoint(self, league):
        steps = self.trained_steps - self._checkpoint_step
        if steps < self.min_steps:
            return False
        hist = league.historical_of()
        wr = league.win_rates(self.pid, hist)
        return (len(wr) > 0 and wr.min() > 0.7) or steps > self.max_steps


ROLES = {"simple": SimplePlayer, "main": MainPlayer, "main_exploiter": MainExploiter,
         "league_exploiter": LeagueExploiter}


def alphastar_roles(world: int, main_agents_n: int = None, main_exploiters_n: int = None,
                    league_exploiters_n: int = 0) -> List[str]:
    """Role of each rank (alpha_star_league.py:23-40): mains first, then main exploiters, then league
    exploiters. Default split for config 4: half main players, half main exploiters."""
    if main_agents_n is None:
        main_agents_n = max(1, world // 2)
    if main_exploiters_n is None:
        main_exploiters_n = world - main_agents_n - league_exploiters_n
    roles = ["main"] * main_agents_n + ["main_exploiter"] * main_exploiters_n + ["league_exploiter"] * league_exploiters_n
    if len(roles) != world:
        raise ValueError(f"{len(roles)} league roles for {world} ranks")
    return roles
