#!/bin/bash
# Round-end evidence at the current tree: counters of MODES (default refil) merged into profiles/counters.json
# (COMMIT names the commit), the whole GPU suite + smoke + the default bench line (gpu_quick.sh), and the default
# `python3 bench.py` under rocprofv3 --kernel-trace --stats (the driver's command).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${MODES-refil}" ]; then
  MODES=${MODES-refil} COMMIT=${COMMIT:-unknown} MERGE=profiles/counters.json bash scripts/gpu_counters.sh \
      > gpurun_out/cnt.log 2>&1 || { tail -20 gpurun_out/cnt.log; exit 1; }
  tail -1 gpurun_out/cnt.log
fi
SMOKE=1 bash scripts/gpu_quick.sh || exit 1
mkdir -p gpurun_out/final_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/final_prof" -o run \
    -- python3 bench.py > gpurun_out/final_prof/bench.json 2> gpurun_out/final_prof/bench.err \
    || { tail -20 gpurun_out/final_prof/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/final_prof/bench.json'))
print('under rocprofv3', round(d['value']/1e6,2), d['roofline']['avg_kernel_ms'], d['league']['value']/1e6, d['refil']['value']/1e6)"
