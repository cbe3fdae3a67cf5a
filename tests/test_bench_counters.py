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


V7_SOURCES = ("ma-league_amd/csrc/rollout.hip", "ma-league_amd/csrc/mlg_device.h", "ma-league_amd/csrc/agent_device.h")


def test_v7_latency_floor_stamp_is_current():
    """the one-env step cycles behind roofline.latency_floor_ms must come from the v7 sources in the
    tree: the recorded stamp commit may not be older than the last commit that changed them (skipped where the tree
    has no git history, e.g. the GPU box's snapshot)."""
    import subprocess
    c = _counters("rollout_v2_kernel<64, true, 5, 10>")
    stamp = c.get("one_env_step_commit")
    assert stamp, "the v7 one-env step cycles name the commit of the sources they were measured on"

    def git(*a):
        return subprocess.run(["git", "-C", ROOT, *a], capture_output=True, text=True)

    if git("rev-parse", "--git-dir").returncode != 0:
        import pytest
        pytest.skip("no git history in this tree")
    last = git("log", "-1", "--format=%H", "--", *V7_SOURCES).stdout.strip()
    assert last, "v7 sources not in the history"
    r = git("merge-base", "--is-ancestor", last, stamp)
    assert r.returncode == 0, (f"v7 sources changed at {last[:7]} after the one-env step stamp ({stamp}): re-measure "
                               "with scripts/gpu_stamps_trace.sh STAMPS=1 and update profiles/counters.json")
    dirty = git("status", "--porcelain", "--", *V7_SOURCES).stdout.strip()
    assert not dirty, f"uncommitted v7 source changes: re-measure the one-env step after committing ({dirty})"
