"""The committed counter evidence bench.py reads into its line (profiles/counters.json): every default-path rollout
kernel has an entry with HBM bytes, and the v7 entry keeps the one-env step cycles the line's latency floor
(roofline.latency_floor_ms) is computed from -- a counter re-collection must not drop them."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _counters(kernel):
    sys.path.insert(0, ROOT)
    import bench
    return bench.load_counters(kernel)


def test_rollout_counters_present():
    for k in ("rollout_v2_kernel<64, true, 5, 10>", "rollout_sp8_kernel<10, 10>", "refil_rollout4_kernel<2, 16>"):
        c = _counters(k)
        assert c.get("hbm_bytes_per_launch", 0) > 0, k
        assert c.get("commit"), k


def test_v7_latency_floor_annotation_present():
    c = _counters("rollout_v2_kernel<64, true, 5, 10>")
    assert c.get("one_env_step_cycles", 0) > 10000
    assert "stamps" in c.get("one_env_step_source", "")
