"""MainLogger parity: the reference's stat keys, aggregation and flush rules.

tests/golden/logger.npz was recorded from the reference MainLogger (src/custom_logging/logger.py:24-173) by
tests/golden/make_golden.py::logger_fixture; the same collect()/log() sequence is replayed here. Every stat
(key, t, value, NaN included) must match, except `steps_mean`: the reference drops the int it is given with
parallel=True (logger.py:135), so its value is always NaN; ours records it (documented fix)."""
import json
import math
from types import SimpleNamespace

import numpy as np

from maleague.custom_logging import Collectibles, MainLogger, Originator


def _replay(lg):
    def run(rets, won_h, won_a, draw, steps):
        lg.collect(Collectibles.RETURN, rets, origin=Originator.HOME, parallel=True)
        lg.collect(Collectibles.WON, won_h, origin=Originator.HOME, parallel=True)
        lg.collect(Collectibles.WON, won_a, origin=Originator.AWAY, parallel=True)
        lg.collect(Collectibles.DRAW, draw, parallel=True)
        lg.collect(Collectibles.STEPS, steps, parallel=True)

    run([1.5, 2.0, -1.0], [True, False, True], [False, True, False], [False, False, False], 37)
    lg.log(0)
    run([0.25], [False], [False], [True], 12)
    lg.log(50)
    # numpy inputs, as the HIP stepper hands them over
    run(np.array([3.0, 4.5]), np.array([True, True]), np.array([False, False]), np.array([False, False]), 20)
    lg.log(150)
    lg.collect(Collectibles.RETURN, 7.0, origin=Originator.HOME)
    lg.collect(Collectibles.WON, True, origin=Originator.HOME)
    lg.collect(Collectibles.DRAW, False)
    lg.log(200)
    lg.test_mode = True
    run([1.0, 2.0], [True, False], [False, False], [False, True], 9)
    lg.log(260)
    run([5.0, 6.0], [False, False], [True, False], [False, False], 9)
    lg.log(260)
    lg.test_mode = False
    lg.log(270)
    lg.log(351)


def test_logger_matches_reference(golden):
    d = golden("logger.npz")
    lg = MainLogger(None, SimpleNamespace(test_nepisode=4, runner_log_interval=100))
    _replay(lg)
    ref = {}
    for i in range(int(d["n"])):
        ref.setdefault(str(d[f"k{i}"]), []).append((int(d[f"t{i}"]), float(d[f"v{i}"])))
    assert sorted(lg.stats) == sorted(ref)
    ours_steps = {"steps_mean": [(0, 37.0), (150, 16.0), (270, math.nan)], "test_steps_mean": [(260, 9.0)]}
    for k, series in ref.items():
        got = [(t, float(v)) for t, v in lg.stats[k]]
        want = ours_steps.get(k, series)
        assert [t for t, _ in got] == [t for t, _ in want], k
        np.testing.assert_allclose([v for _, v in got], [v for _, v in want], rtol=1e-12, equal_nan=True, err_msg=k)


def test_logger_sinks(tmp_path):
    run = SimpleNamespace(info={})
    lg = MainLogger(None, SimpleNamespace(test_nepisode=2, runner_log_interval=10))
    lg.setup_json(str(tmp_path))
    lg.setup_sacred(run)
    lg.collect(Collectibles.RETURN, [1.0, 3.0], parallel=True)
    lg.log(5)
    lg.log_stat("home_qlearner_loss", 0.5, 7)
    lines = [json.loads(x) for x in open(tmp_path / "stats.jsonl")]
    by_key = {x["key"]: x for x in lines}
    assert by_key["home_return_mean"] == {"key": "home_return_mean", "t": 5, "value": 2.0}
    assert by_key["away_return_mean"]["value"] is None  # NaN -> null
    assert "home_actions_taken_extract_greedy_actions" not in by_key  # image stats are not scalars
    assert run.info["home_return_mean"] == [2.0] and run.info["home_return_mean_T"] == [5]
    assert run.info["home_qlearner_loss"] == [0.5]


def test_console_report(caplog):
    lg = MainLogger(console=True, log_interval=1)
    lg.log_stat("episode", 8, 100)
    for i in range(7):
        lg.log_stat("home_return_mean", float(i), 100 + i)
    with caplog.at_level("INFO", logger="maleague"):
        lg.log_report()
    assert "Recent Stats | t_env:        100 | Episode:        8" in caplog.text
    assert "{:<25}{:>8}".format("home_return_mean:", "4.0000") in caplog.text  # mean of the last 5 values
