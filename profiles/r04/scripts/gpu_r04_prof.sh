#!/bin/bash
# Round-4 profile: per mode, rocprofv3 --kernel-trace --stats of a short bench (timeline of the timed iterations via
# scripts/trace_iter.py), then the counter passes of scripts/gpu_counters.sh (rollout + learner kernels).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${MODES:-ai league refil}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/trace_$m" -o run \
      -- python3 bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace_$m.json 2> gpurun_out/trace_$m.err \
      || { echo "trace $m failed"; tail -20 gpurun_out/trace_$m.err; exit 1; }
  key=$( [ $m = ai ] && echo rollout_v2_kernel || ( [ $m = league ] && echo rollout_sp7 || echo refil_rollout ) )
  python3 scripts/trace_iter.py gpurun_out/trace_$m/run_kernel_trace.csv $key 6 > gpurun_out/trace_$m.txt || exit 1
  head -30 gpurun_out/trace_$m.txt
done
[ -n "$NO_COUNTERS" ] && exit 0
COMMIT=${COMMIT:-unknown} bash scripts/gpu_counters.sh > gpurun_out/counters.log 2>&1 || { tail -20 gpurun_out/counters.log; exit 1; }
tail -3 gpurun_out/counters.log
