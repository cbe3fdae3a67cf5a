#!/bin/bash
# Timing diagnostic (wrong results by design): sp8 stamps when only waves 0-3 run the env step -- how much of the env
# phase is contention between the two waves of a SIMD vs one wave's latency. The library was a one-off build (not in
# the tree): rollout_sp8.inc with the env step calls (sp_lane_step1 / step2 / sp8_obs_pad) wrapped in
# `if (wave < 4) { ... }`, compiled with -DMLG_STAMPS into _lib/variants/stamps_halfenv.so (scripts/build_variant.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/stamps
export SP_RS=16 SP_SLOTS=fc1,bar_fc1,x_planes,bar_x,gru,bar_gru,h_planes,bar_h,fc2,bar_fc2,env_step1,env_step2,tail,bar_env,rowmap
MLG_LIB=ma-league_amd/maleague/_lib/variants/stamps_halfenv.so timeout -k 10 300 python scripts/stamps_sp.py \
  > gpurun_out/stamps/sp8_halfenv.txt 2>&1 || { echo "halfenv stamps failed"; tail -20 gpurun_out/stamps/sp8_halfenv.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps/sp8_halfenv.txt | head -40
