#!/bin/bash
# GPU tests (learners), then rocprofv3 kernel stats of bench (ai) and bench (refil). Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_learner.py tests/test_gpu_refil_learner.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/l.log 2>&1 || { tail -30 gpurun_out/l.log; exit 1; }
tail -2 gpurun_out/l.log
export TMPDIR=/tmp
for m in ai refil; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$m" -o run -- python bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$m.json 2> gpurun_out/prof_$m.err || { echo "rocprof $m failed"; tail -20 gpurun_out/prof_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/prof_$m.json')); print('$m', d['value']/1e6, 'M env-steps/s', d['ms_per_step'], 'ms/step')"
  python scripts/prof_top.py gpurun_out/prof_$m/run_kernel_stats.csv 12
done
