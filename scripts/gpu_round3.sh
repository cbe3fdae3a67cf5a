#!/bin/bash
# Round-3 check on the GPU box: all GPU tests + smoke, the default bench (config 2 + league leg + CPU baselines),
# then each mode under rocprofv3 --kernel-trace --stats. Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); L=d['league']; print('ai', d['value']/1e6, d['ms_per_step'], 'frac', d['roofline']['frac'], '| league', L['value']/1e6, L['ms_per_step'], 'exch', L['exchange_ms_mean'], '| cpu', [round(x['value']) for x in d['cpu_baseline']['legs']])"
export TMPDIR=/tmp
for m in ${MODES:-ai league refil}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$m" -o run \
      -- python bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$m.json 2> gpurun_out/prof_$m.err \
      || { echo "rocprof $m failed"; tail -20 gpurun_out/prof_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/prof_$m.json')); print('$m', d['value']/1e6, 'M env-steps/s', d['ms_per_step'], 'ms/step', 'kernel', d['roofline']['avg_kernel_ms'])"
  python scripts/prof_top.py gpurun_out/prof_$m/run_kernel_stats.csv 6
done
