#!/bin/bash
# v7 rollout phase stamps (diagnostic builds): all steps, sparse steps (<= 2 envs running in the workgroup) and the
# timeline of the first one-env step.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/stamps
for v in all:ma-league_amd/maleague/_lib/libmaleague_stamps.so low:ma-league_amd/maleague/_lib/variants/stampslow.so \
         tl:ma-league_amd/maleague/_lib/variants/stampstl.so full:ma-league_amd/maleague/_lib/variants/stampsfull.so; do
  name=${v%%:*}; lib=${v#*:}
  MINRUN=$([ $name = full ] && echo 16 || echo 0) TIMELINE=$([ $name = tl ] && echo 1 || echo 0) MLG_ROLLOUT_KERNEL=v7 MLG_LIB=$lib timeout -k 10 300 \
      python scripts/stamps_rollout.py > gpurun_out/stamps/$name.txt 2>&1 || { echo "stamps $name failed"; tail -20 gpurun_out/stamps/$name.txt; exit 1; }
  echo "== $name"; grep -v amdgpu.ids gpurun_out/stamps/$name.txt | grep -v "slowest WG steps" | head -45
done
MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 300 python scripts/stamps_refil.py \
    > gpurun_out/stamps/refil.txt 2>&1 || { echo "stamps refil failed"; tail -20 gpurun_out/stamps/refil.txt; exit 1; }
echo "== refil"; grep -v amdgpu.ids gpurun_out/stamps/refil.txt | head -30
