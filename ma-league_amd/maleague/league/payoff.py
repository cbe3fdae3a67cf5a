"""Payoff table and PFSP/FSP opponent sampling (src/league/components/payoff_entry.py:7-51,
self_play.py:17-72), host side.

Differences from the reference, all listed in SURVEY Appendix A:
* ``record_result`` increments GAMES together with WIN/LOSS/DRAW -- the reference never increments GAMES,
  so its win rates are always 0.5 and PFSP degenerates to uniform; ``reference_compat=True`` reproduces that.
* FSP samples uniformly (the reference passes a scalar ``p`` to np.random.choice, self_play.py:35-37).
* PFSP with a vanishing norm samples uniformly (the reference returns a probability array, :61-63).
"""
from __future__ import annotations

from enum import IntEnum

import numpy as np
import torch


class PayoffEntry(IntEnum):
    GAMES = 0
    WIN = 1
    LOSS = 2
    DRAW = 3
    MATCHES = 4


class PayoffWrapper:
    def __init__(self, payoff: torch.Tensor, reference_compat: bool = False):
        self._p = payoff
        self.reference_compat = reference_compat

    @property
    def tensor(self):
        return self._p

    def win_rates(self, idx, indices=None):
        row = self._p[idx] if indices is None else self._p[idx, indices]
        games = row[:, PayoffEntry.GAMES]
        wr = (row[:, PayoffEntry.WIN] + 0.5 * row[:, PayoffEntry.DRAW]) / games
        wr[games == 0.0] = 0.5
        return wr

    def games(self, i):
        return self._p[i, :, PayoffEntry.GAMES]

    def matches(self, i):
        return self._p[i, :, PayoffEntry.MATCHES]

    def increment(self, i, j, entry: PayoffEntry, n=1):
        self._p[i, j, entry] += n

    def win(self, i, j):
        self.increment(i, j, PayoffEntry.WIN)

    def draw(self, i, j):
        self.increment(i, j, PayoffEntry.DRAW)

    def loss(self, i, j):
        self.increment(i, j, PayoffEntry.LOSS)

    def match(self, i, j):
        self.increment(i, j, PayoffEntry.MATCHES)

    def record_result(self, i, j, result: PayoffEntry, n=1):
        """One finished episode of home i vs away j (league_experiment_process.py:85-105)."""
        self.increment(i, j, result, n)
        if not self.reference_compat:
            self.increment(i, j, PayoffEntry.GAMES, n)


def episode_result(env_info, policy_team_id=0) -> PayoffEntry:
    """_extract_result (league_experiment_process.py:85-95): draw if the env says so or if both/no team won."""
    won = env_info["battle_won"]
    if env_info.get("draw", False) or all(won) or not any(won):
        return PayoffEntry.DRAW
    return PayoffEntry.WIN if won[policy_team_id] else PayoffEntry.LOSS


WEIGHTINGS = {
    "variance": lambda x: x * (1 - x),
    "linear": lambda x: 1 - x,
    "linear_capped": lambda x: np.minimum(0.5, 1 - x),
    "squared": lambda x: (1 - x) ** 2,
}


class PFSPSampling:
    def __init__(self, rng: np.random.RandomState | None = None):
        self.rng = rng or np.random

    def probabilities(self, prio_measure, weighting="linear"):
        w = WEIGHTINGS[weighting](np.asarray(prio_measure, dtype=np.float64))
        norm = w.sum()
        if norm < 1e-10:
            return np.ones_like(w) / len(w)
        return w / norm

    def sample(self, opponents, prio_measure=None, weighting="linear"):
        if prio_measure is None:
            raise Exception("Please serve up-to-date prioritization measure.")
        p = self.probabilities(prio_measure, weighting)
        return opponents[self.rng.choice(len(opponents), p=p)]


class FSPSampling:
    def __init__(self, rng: np.random.RandomState | None = None):
        self.rng = rng or np.random

    def sample(self, opponents):
        return opponents[self.rng.randint(len(opponents))]


class SPSampling:
    def __init__(self, opponent_id):
        self.opponent_id = opponent_id

    def sample(self, opponents):
        return opponents[self.opponent_id]


REGISTRY = {"sp": SPSampling, "fsp": FSPSampling, "pfsp": PFSPSampling}
