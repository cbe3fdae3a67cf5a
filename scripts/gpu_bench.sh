#!/bin/bash
# Round benchmark + rocprofv3 kernel-trace summary on the GPU box. Each GPU step has its own timeout;
# steps are chained so that a failure stops the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
STEPS=${STEPS:-20}
timeout -k 10 900 python bench.py --steps "$STEPS" --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof failed rc=$?"; exit 1; }
find gpurun_out/prof -name "*stats*" | head
