#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TIMELINE=1 MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/variants/stampstl.so timeout -k 10 300 \
    python scripts/stamps_rollout.py > gpurun_out/stampstl.txt 2>&1 || { echo "stamps tl failed"; tail -20 gpurun_out/stampstl.txt; exit 1; }
grep "timeline" gpurun_out/stampstl.txt
