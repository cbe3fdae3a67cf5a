#!/bin/bash
# wgrad chunking sweep: config-2 bench line per MLG_WGRAD_WAVES value, plus the wgrad kernel times under rocprofv3.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WAVES:-128 256 512}; do
  MLG_WGRAD_WAVES=$w timeout -k 10 300 python bench.py --mode ai --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sw_$w.json 2> gpurun_out/sw_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/sw_$w.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sw_$w.json')); print('waves $w', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), 'ms/step')"
  MLG_WGRAD_WAVES=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/sw_prof_$w" -o run \
      -- python bench.py --mode ai --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/sw_prof_$w.err || { echo "rocprof $w failed"; exit 1; }
  python scripts/prof_top.py gpurun_out/sw_prof_$w/run_kernel_stats.csv 12 | grep wgrad
done
