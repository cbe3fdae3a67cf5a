#!/bin/bash
# REFIL dev session: REFIL GPU tests, then the rollout microbenchmark. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_refil.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/refil_tests.log 2>&1
rc=$?
tail -30 gpurun_out/refil_tests.log
[ $rc -eq 0 ] || { echo "refil tests failed rc=$rc"; exit 1; }
timeout -k 10 300 python scripts/bench_refil_rollout.py > gpurun_out/refil_rollout.txt 2>&1 || { echo "bench failed"; cat gpurun_out/refil_rollout.txt; exit 1; }
cat gpurun_out/refil_rollout.txt
