#!/bin/bash
# Round check on the GPU box: all GPU tests, then bench (ai = config 2, league = config 3/4 on one GPU,
# refil = config 5) each under rocprofv3 --kernel-trace --stats. Every step has its own time limit and the
# script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
for m in ${MODES:-ai league refil}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$m" -o run \
      -- python bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$m.json 2> gpurun_out/prof_$m.err \
      || { echo "rocprof $m failed"; tail -20 gpurun_out/prof_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/prof_$m.json')); print('$m', d['value']/1e6, 'M env-steps/s', d['ms_per_step'], 'ms/step')"
  python scripts/prof_top.py gpurun_out/prof_$m/run_kernel_stats.csv 8
done
