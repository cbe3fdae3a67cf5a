#!/bin/bash
# v7 one-env step cycles at HEAD (stamps build, STAMPS=1) and per-iteration kernel timelines of the bench legs
# (MODES, rocprofv3 --kernel-trace --stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$STAMPS" ]; then
  MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 300 \
      python scripts/stamps_rollout.py > gpurun_out/stamps_v7.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps_v7.txt; exit 1; }
  grep -E "nrun= 1|nrun=16|per-WG|episode len" gpurun_out/stamps_v7.txt
fi
for m in ${MODES:-}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/trace_$m" -o run \
      -- python3 bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace_$m.json 2> gpurun_out/trace_$m.err \
      || { echo "trace $m failed"; tail -20 gpurun_out/trace_$m.err; exit 1; }
  key=$( [ $m = ai ] && echo rollout_v2_kernel || ( [ $m = league ] && echo rollout_sp || echo refil_rollout ) )
  python3 scripts/trace_iter.py gpurun_out/trace_$m/run_kernel_trace.csv $key 6 > gpurun_out/trace_$m.txt || exit 1
  head -${TRACE_LINES:-30} gpurun_out/trace_$m.txt
done
