#!/bin/bash
# Phase stamps of both rollout kernels (diagnostic build).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for k in ${KERNELS:-v1 v2}; do
  MLG_ROLLOUT_KERNEL=$k MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 300 python scripts/stamps_rollout.py > gpurun_out/stamps_$k.txt 2>&1 || { echo "stamps $k failed"; cat gpurun_out/stamps_$k.txt; exit 1; }
  echo "== $k"; grep -v amdgpu.ids gpurun_out/stamps_$k.txt
done
