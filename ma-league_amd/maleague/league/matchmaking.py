"""Matchmakers of the matchmaking league (src/league/components/matchmaker.py:16-150), over the replicated
league state instead of a queue to the agent-pool process.

Every ``get_match(home_pid, league)`` returns the opponent pid (a learning player; historical snapshots are
the role-based players' business) or None when the league is over for this player, and records the match
(``payoff.match``, matchmaker.py:71) into the caller's local payoff delta through ``record_match``.
"""
from __future__ import annotations

import numpy as np

from .payoff import PayoffEntry, PFSPSampling


class Matchmaker:
    def __init__(self, rng=None, record_match=None):
        self.rng = rng or np.random.RandomState(0)
        self.record_match = record_match or (lambda i, j: None)

    def get_match(self, home, league):
        raise NotImplementedError()

    def _matched(self, home, chosen):
        self.record_match(home, chosen)
        return chosen


class PFSPMatchmaking(Matchmaker):
    """matchmaker.py:64-72: PFSP (linear weighting) over every agent of the pool, self included."""

    def __init__(self, rng=None, record_match=None, weighting="linear"):
        super().__init__(rng, record_match)
        self._sampling = PFSPSampling(self.rng)
        self.weighting = weighting

    def get_match(self, home, league):
        opponents = [p.pid for p in league.players]
        wr = league.win_rates(home, opponents)
        return self._matched(home, int(self._sampling.sample(opponents, prio_measure=wr, weighting=self.weighting)))


class FSPMatchmaking(Matchmaker):
    """matchmaker.py:75-86 (uniform; the reference's scalar ``p`` to np.random.choice is a defect)."""

    def get_match(self, home, league):
        opponents = [p.pid for p in league.players]
        return self._matched(home, opponents[self.rng.randint(len(opponents))])


class BalancedMatchmaking(Matchmaker):
    """matchmaker.py:89-101: the opponent played the least (argmin of MATCHES, first on ties)."""

    def get_match(self, home, league):
        n = len(league.players)
        matches = league.payoff.tensor[home, :n, PayoffEntry.MATCHES].detach().cpu()
        return self._matched(home, int(matches.argmin().item()))


class RandomMatchmaking(Matchmaker):
    """matchmaker.py:104-118."""

    def get_match(self, home, league):
        return self._matched(home, int(self.rng.randint(len(league.players))))


class NonRecurringAllAdversaryMatchmaking(Matchmaker):
    """matchmaker.py:121-141: every other player once, never self; None when all were played."""

    def get_match(self, home, league):
        n = len(league.players)
        matches = league.payoff.tensor[home, :n, PayoffEntry.MATCHES].detach().cpu().clone()
        matches[home] = 2
        if bool((matches > 0).all()):
            return None
        chosen = int(matches.argmin().item())
        assert chosen != home
        return self._matched(home, chosen)


REGISTRY = {"pfsp": PFSPMatchmaking, "uniform": BalancedMatchmaking, "random": RandomMatchmaking,
            "fsp": FSPMatchmaking, "adversaries": NonRecurringAllAdversaryMatchmaking}
