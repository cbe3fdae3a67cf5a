#!/bin/bash
# REFIL rollout phase stamps (diagnostic build): phase shares, per-step cost by number of running pairs, the
# critical (slowest) wave.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/stamps
LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so
MLG_LIB=$LIB timeout -k 10 300 python scripts/stamps_refil.py > gpurun_out/stamps/refil.txt 2>&1 \
  || { echo "stamps refil failed"; tail -20 gpurun_out/stamps/refil.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps/refil.txt | head -90
