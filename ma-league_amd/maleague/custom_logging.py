"""MainLogger with the reference's collect/log/log_stat surface and stat keys (src/custom_logging/logger.py:24-173,
collectibles.py:10-68, utils/preprocessing.py, platforms/console.py:25-54).

Aggregation follows the reference: per collectible, global ones (DRAW, STEPS) log `{prefix}{name}_{fn}`, the others
`{prefix}{origin}_{name}_{fn}` for both origins (home, away), NaN when nothing was collected; train stats are flushed
every `runner_log_interval` env steps, test stats once `test_nepisode` home returns were collected
(`logger.py:69-84, 103-122`). Pinned by tests/golden/logger.npz (recorded from the reference).

Deliberate difference: `collect(..., parallel=True)` also accepts numpy arrays and scalars (the reference keeps
only Python lists, so its `steps_mean` -- collected as an int -- is always NaN; SURVEY Appendix A style fix).

Sinks without sacred: `setup_json(log_dir)` (one JSON object per stat line, `stats.jsonl`), `setup_sacred(run)`
(any object with an `info` dict, same `{key}` / `{key}_T` lists as CustomSacredLogger), `setup_tensorboard(log_dir)`
(torch.utils.tensorboard; raises ImportError when the tensorboard package is absent)."""
from __future__ import annotations

import json
import logging
import math
import os
from collections import defaultdict
from enum import Enum

import numpy as np


class Originator(str, Enum):
    HOME = "home"
    AWAY = "away"

    @classmethod
    def list(cls):
        return [c.value for c in cls]


def percentage(x):
    """utils/preprocessing.py: share of truthy entries."""
    return np.sum(np.array(x, dtype=int), axis=0) / len(x)


def extract_greedy_actions(episodal_actions_taken):
    """utils/preprocessing.py: per agent, the actions taken greedily. Input: list of [t, 2, n_agents] arrays
    (row 0 actions, row 1 is-greedy flags)."""
    if len(episodal_actions_taken) == 0:
        return []
    a = np.concatenate([np.asarray(x) for x in episodal_actions_taken], axis=0)
    greedy = a[:, 1, :] == 1
    return [a[:, 0, i][greedy[:, i]].tolist() for i in range(a.shape[-1])]


class Collectibles(Enum):
    """collectibles.py:10-41: (preprocessing, log_type, is_global)."""
    RETURN = ((np.mean, np.std), "scalar", False)
    ACTIONS_TAKEN = ((extract_greedy_actions,), "image", False)
    WON = ((percentage,), "scalar", False)
    DRAW = ((percentage,), "scalar", True)
    STEPS = ((np.mean,), "scalar", True)

    @property
    def preprocessing(self):
        return self.value[0]

    @property
    def log_type(self):
        return self.value[1]

    @property
    def is_global(self):
        return self.value[2]

    @property
    def keys(self):
        return [f"{self.name.lower()}_{p.__name__}" for p in self.preprocessing]


class _JsonSink:
    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, "stats.jsonl")
        self._f = open(self.path, "a", buffering=1)

    def log(self, key, value, t, log_type):
        if log_type != "scalar":
            return
        v = float(value)
        self._f.write(json.dumps({"key": key, "t": int(t), "value": None if math.isnan(v) else v}) + "\n")


class _SacredSink:
    """platforms/sacred.py: appends to run.info[key] / run.info[key + '_T']."""

    def __init__(self, run):
        self.info = run.info

    def log(self, key, value, t, log_type):
        if log_type != "scalar":
            return
        if key in self.info:
            self.info[f"{key}_T"].append(t)
            self.info[key].append(value)
        else:
            self.info[f"{key}_T"] = [t]
            self.info[key] = [value]


class _TensorboardSink:
    def __init__(self, log_dir):
        from torch.utils.tensorboard import SummaryWriter  # needs the tensorboard package
        self.writer = SummaryWriter(log_dir=log_dir)

    def log(self, key, value, t, log_type):
        if log_type == "scalar":
            self.writer.add_scalar(key, float(value), t)


class _Chunk:
    __slots__ = ("a",)

    def __init__(self, a):
        self.a = a


class _Series:
    """One collectible's episodal values: scalar appends and whole per-run arrays, the arrays kept as arrays until the
    stats are computed at log time (a list of 4096 Python floats per run and collectible cost ~0.1 ms of host time per
    training iteration). values() is the reference's list, in collection order."""
    __slots__ = ("_items", "_n")

    def __init__(self):
        self._items, self._n = [], 0

    def append(self, v):
        self._items.append(v)
        self._n += 1

    def extend_array(self, a):
        """Arrays are copied (a caller changing its array in place later must not change unlogged stats); lists and
        tuples stay Python values, extended as the reference's list.extend does (no dtype coercion)."""
        if isinstance(a, (list, tuple)):
            self._items.extend(a)
            self._n += len(a)
            return
        a = np.array(a, copy=True).reshape(-1)
        self._items.append(_Chunk(a))
        self._n += a.size

    def clear(self):
        self._items.clear()
        self._n = 0

    def __len__(self):
        return self._n

    def values(self) -> list:
        out = []
        for x in self._items:
            if type(x) is _Chunk:
                out.extend(x.a.tolist())
            else:
                out.append(x)
        return out


class MainLogger:
    """`MainLogger(console_logger, args)` as in the reference; `console=` / `log_interval=` are shorthands for
    callers without an args namespace (runner_log_interval, test_nepisode default 2000 / 0)."""

    def __init__(self, console_logger=None, args=None, console=False, log_interval=None):
        self.args = args
        self.console = console or console_logger is not None
        self._console = console_logger if console_logger is not None else logging.getLogger("maleague")
        self.stats = defaultdict(list)
        self.test_mode = False
        self.test_n_episode = int(getattr(args, "test_nepisode", 0) or 0)
        self.runner_log_interval = (log_interval if log_interval is not None
                                    else int(getattr(args, "runner_log_interval", 2000)))
        self.log_interval = self.runner_log_interval
        self.log_train_stats_t = -1000000  # log the first run (logger.py:45)
        self._sinks = []
        self.episodal_stats = {c: {m: (_Series() if c.is_global else {o: _Series() for o in Originator.list()})
                                   for m in ("train", "test")} for c in Collectibles}

    @classmethod
    def from_args(cls, args, log_dir=None):
        """The run setup of the reference (console + TensorBoard when `use_tensorboard`), with a JSON-lines sink
        under `log_dir` standing in for sacred's file observer."""
        lg = cls(logging.getLogger("maleague"), args)
        if log_dir is not None:
            lg.setup_json(log_dir)
            if getattr(args, "use_tensorboard", False):
                lg.setup_tensorboard(os.path.join(log_dir, "tb_logs"))
        return lg

    # -- sinks -----------------------------------------------------------------------------------------------
    def setup_json(self, log_dir):
        self._sinks.append(_JsonSink(log_dir))

    def setup_sacred(self, sacred_run_dict):
        self._sinks.append(_SacredSink(sacred_run_dict))

    def setup_tensorboard(self, log_dir):
        self._sinks.append(_TensorboardSink(log_dir))

    def update_scheme(self, scheme):
        self.scheme = scheme

    def info(self, msg):
        if self.console:
            self._console.info(msg)

    def error(self, msg):
        self._console.error(msg)

    # -- collection ------------------------------------------------------------------------------------------
    def _bucket(self, collectible, origin):
        stat = self.episodal_stats[collectible]["test" if self.test_mode else "train"]
        return stat if collectible.is_global else stat[Originator(origin).value]

    def collect(self, collectible: Collectibles, data, origin: Originator = Originator.HOME, parallel=False):
        """logger.py:124-146. parallel=True extends by the entries of `data`; otherwise appends it."""
        bucket = self._bucket(collectible, origin if origin is not None else Originator.HOME)
        if parallel and isinstance(data, (list, tuple, np.ndarray)):
            bucket.extend_array(data)
        else:
            bucket.append(data.item() if isinstance(data, np.generic) else data)

    def preprocess_collectible(self, collectible: Collectibles, origin=None):
        data = self._bucket(collectible, origin if origin is not None else Originator.HOME).values()
        return [fn(data) if len(data) > 0 else np.nan for fn in collectible.preprocessing]

    def log(self, t_env):
        """logger.py:69-84: test stats once the test episodes are complete, train stats per interval."""
        test_returns = self.episodal_stats[Collectibles.RETURN]["test"][Originator.HOME.value]
        if self.test_mode and len(test_returns) == self.test_n_episode:
            self._log_collectibles(t_env)
        elif not self.test_mode and t_env - self.log_train_stats_t >= self.runner_log_interval:
            self._log_collectibles(t_env)
            self.log_train_stats_t = t_env

    def _log_collectibles(self, t_env):
        mode = "test" if self.test_mode else "train"
        prefix = "test_" if self.test_mode else ""
        for c in Collectibles:
            if c.is_global:
                for k, v in zip(c.keys, self.preprocess_collectible(c)):
                    self.log_stat(f"{prefix}{k}", v, t_env, log_type=c.log_type)
                self.episodal_stats[c][mode].clear()
            else:
                for origin in Originator.list():
                    for k, v in zip(c.keys, self.preprocess_collectible(c, origin)):
                        self.log_stat(f"{prefix}{origin}_{k}", v, t_env, log_type=c.log_type)
                    self.episodal_stats[c][mode][origin].clear()

    def log_stat(self, key, value, t, log_type="scalar", to_sacred=True):
        self.stats[key].append((t, value))
        for sink in self._sinks:
            sink.log(key, value, t, log_type)

    def log_report(self):
        """platforms/console.py:25-54: mean of the last 5 values per stat (1 for epsilon), 4 per line."""
        if not self.console or "episode" not in self.stats:
            return
        s = "Recent Stats | t_env: {:>10} | Episode: {:>8}\n".format(*self.stats["episode"][-1])
        i = 0
        for key in sorted(self.stats):
            if key == "episode" or "actions_taken_extract_greedy_actions" in key:
                continue
            i += 1
            window = 1 if key == "epsilon" else 5
            s += "{:<25}{:>8}".format(key + ":", "{:.4f}".format(np.mean([float(x[1]) for x in self.stats[key][-window:]])))
            s += "\n" if i % 4 == 0 else "\t"
        self._console.info(s)
