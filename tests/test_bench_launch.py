"""bench.py's own multi-rank launch (the way the driver invokes it: ``python bench.py --gpus N``, no outer
torch.distributed.run). The parent must start N ranks itself, relay rank 0's single JSON line and fail when a rank
fails. ``--dry-run --backend gloo`` runs the same launcher and process-group code on CPU, plus one league exchange
(payoff all_reduce, parameter all_gather, barrier) over the launched group."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 4, 8])  # 8: the driver's full-node run
def test_bench_gpus_n_self_launches_n_ranks(n):
    p = _bench("--gpus", str(n), "--backend", "gloo", "--dry-run")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = p.stdout.strip().splitlines()
    assert len(lines) == 1, p.stdout  # stdout carries exactly the JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["dry_run"] is True
    assert out["ranks"] == list(range(n))
    lg = out["league"]
    assert lg["world_size"] == n and lg["collective_backend"] == "gloo"
    assert lg["params_of"] == [float(r) for r in range(n)]  # every rank's vector gathered
    assert lg["payoff_wins"] == sum(r + 1 for r in range(n))  # every rank's delta reduced
    assert lg["historical_snapshots"] == n


def test_bench_launch_fails_when_a_rank_fails():
    p = _bench("--gpus", "2", "--backend", "no-such-backend", "--dry-run")
    assert p.returncode != 0
    assert p.stdout.strip() == ""


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert p.returncode != 0 and "--gpus 2" in p.stderr
