"""Minimal MainLogger with the reference's collect/log/log_stat surface (src/custom_logging/logger.py:24-173,
collectibles.py:10-68). Stats are kept in memory (``stats[key] -> [(t, value)]``) and optionally echoed
to the console; sacred/TensorBoard sinks are outside the hot path and not built."""
from __future__ import annotations

import logging
from collections import defaultdict
from enum import Enum

import numpy as np


class Originator(str, Enum):
    HOME = "home"
    AWAY = "away"


class Collectibles(Enum):
    RETURN = "return"
    ACTIONS_TAKEN = "actions_taken"
    WON = "won"
    DRAW = "draw"
    STEPS = "steps"


_AGG = {  # collectible -> preprocessing applied at log time (collectibles.py:10-41)
    Collectibles.RETURN: [("mean", np.mean), ("std", np.std)],
    Collectibles.WON: [("percentage", lambda v: float(np.mean(np.asarray(v, dtype=np.float64))) if len(v) else 0.0)],
    Collectibles.DRAW: [("percentage", lambda v: float(np.mean(np.asarray(v, dtype=np.float64))) if len(v) else 0.0)],
    Collectibles.STEPS: [("mean", np.mean)],
}


class MainLogger:
    def __init__(self, console=False, log_interval=2000):
        self.console = console
        self.test_mode = False
        self.log_interval = log_interval
        self.stats = defaultdict(list)
        self._buf = defaultdict(list)
        self._last_log_t = -log_interval - 1
        self._log = logging.getLogger("maleague")

    def update_scheme(self, scheme):
        self.scheme = scheme

    def collect(self, key: Collectibles, data, origin: Originator = None, parallel=False):
        name = (("test_" if self.test_mode else "") + (f"{origin.value}_" if origin is not None else "") + key.value)
        if parallel and isinstance(data, (list, tuple, np.ndarray)):
            self._buf[(key, name)].append(np.asarray(data))
        else:
            self._buf[(key, name)].append(np.asarray([data]))

    def log(self, t_env):
        if t_env - self._last_log_t < self.log_interval:
            return
        for (key, name), chunks in self._buf.items():
            values = np.concatenate(chunks) if chunks else np.zeros(0)
            for suffix, fn in _AGG.get(key, []):
                if len(values):
                    self.log_stat(f"{name}_{suffix}", float(fn(values)), t_env)
        self._buf.clear()
        self._last_log_t = t_env

    def log_stat(self, key, value, t, to_sacred=True):
        self.stats[key].append((t, value))
        if self.console:
            self._log.info("%s: %s @ %s", key, value, t)

    def log_report(self):
        if self.console:
            for k, v in sorted(self.stats.items()):
                self._log.info("%s %s", k, v[-1])

    def info(self, msg):
        if self.console:
            self._log.info(msg)
