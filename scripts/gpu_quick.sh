#!/bin/bash
# Quick GPU check: rollout tests + deterministic rollout microbenchmark of the given kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_rollout.py -x -q -p no:cacheprovider > gpurun_out/tests_quick.log 2>&1
rc=$?
tail -3 gpurun_out/tests_quick.log
[ $rc -eq 0 ] || { grep -E "^E |Error|assert" gpurun_out/tests_quick.log | head -20; exit 1; }
MLG_BENCH_KERNELS=${KERNELS:-v2,v4} timeout -k 10 300 python scripts/bench_rollout.py
