#!/bin/bash
# REFIL rollout v4 check: REFIL GPU tests (both kernels), fixed-policy timing of both, stamps of v4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_refil.py tests/test_gpu_refil_learner.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/refil_tests.log 2>&1 || { tail -40 gpurun_out/refil_tests.log; exit 1; }
tail -3 gpurun_out/refil_tests.log
for v in v4 v1; do
  MLG_REFIL_ROLLOUT=$v timeout -k 10 120 python scripts/bench_refil_rollout.py > gpurun_out/refil_ro_$v.txt 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/refil_ro_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/refil_ro_$v.txt)"
done
if [ -f ma-league_amd/maleague/_lib/libmaleague_stamps.so ]; then
  MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 120 python scripts/stamps_refil.py > gpurun_out/refil_stamps4.txt 2>&1 && cat gpurun_out/refil_stamps4.txt
fi
