#!/bin/bash
# Self-play rollout phase stamps (diagnostic build): sp8 (16 envs per workgroup) and sp7 for comparison.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/stamps
LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so
SP_RS=16 SP_SLOTS=fc1,bar_fc1,x_planes,bar_x,gru,bar_gru,h_planes,bar_h,fc2,bar_fc2,env_step1,env_step2,tail,bar_env,rowmap \
  MLG_LIB=$LIB timeout -k 10 300 python scripts/stamps_sp.py > gpurun_out/stamps/sp8.txt 2>&1 \
  || { echo "stamps sp8 failed"; tail -20 gpurun_out/stamps/sp8.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps/sp8.txt | head -60
