#!/bin/bash
# GPU session: parity tests, then bench + rocprof (scripts/gpu_bench.sh). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?
tail -5 gpurun_out/tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
bash scripts/gpu_bench.sh
