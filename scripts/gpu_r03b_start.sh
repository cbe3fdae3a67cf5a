#!/bin/bash
# Session start: GPU suite at HEAD, full-occupancy phase stamps of the v7 rollout, fixed-policy rollout timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
MINRUN=16 MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/variants/stamps16.so timeout -k 10 300 \
    python scripts/stamps_rollout.py > gpurun_out/stamps16.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps16.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps16.txt | head -48
RING=1 timeout -k 10 200 python scripts/bench_rollout.py > gpurun_out/ro_default.json 2>/dev/null || { echo "bench failed"; exit 1; }
cat gpurun_out/ro_default.json
