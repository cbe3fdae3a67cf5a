#!/bin/bash
# v7 iteration: rollout / self-play / episode GPU tests, fixed-policy rollout timing (2 reps), full-occupancy stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_episode.py tests/test_gpu_selfplay.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_ro.log 2>&1 || { tail -40 gpurun_out/tests_ro.log; exit 1; }
tail -1 gpurun_out/tests_ro.log
for rep in 1 2; do
  RING=1 timeout -k 10 200 python scripts/bench_rollout.py > gpurun_out/ro_$rep.json 2>/dev/null || { echo "bench failed"; exit 1; }
  cat gpurun_out/ro_$rep.json
done
if [ -e ma-league_amd/maleague/_lib/variants/stamps16.so ]; then
MINRUN=16 MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/variants/stamps16.so timeout -k 10 300 \
    python scripts/stamps_rollout.py > gpurun_out/stamps16.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps16.txt; exit 1; }
grep -A16 "steps with >=" gpurun_out/stamps16.txt; grep "nrun= 1 \|nrun=16" gpurun_out/stamps16.txt
fi
