#!/bin/bash
# Phase stamps of the v7 rollout: full-occupancy steps (stamps16) and the first one-env step timeline (stampstl).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MINRUN=16 MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/variants/stamps16.so timeout -k 10 300 \
    python scripts/stamps_rollout.py > gpurun_out/stamps16.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps16.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps16.txt | grep -v "slowest WG steps" | head -50
TIMELINE=1 MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/variants/stampstl.so timeout -k 10 300 \
    python scripts/stamps_rollout.py > gpurun_out/stampstl.txt 2>&1 || { echo "stamps tl failed"; tail -20 gpurun_out/stampstl.txt; exit 1; }
grep "timeline" gpurun_out/stampstl.txt
