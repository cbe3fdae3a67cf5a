#!/bin/bash
# Rollout tests (QMIX + self-play), rollout microbench, bench ai + league lines.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_selfplay.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_spill.log 2>&1
rc=$?; tail -3 gpurun_out/tests_spill.log
[ $rc -eq 0 ] || { grep -E "^E |Error|assert" gpurun_out/tests_spill.log | head -20; exit 1; }
MLG_BENCH_KERNELS=v2 timeout -k 10 300 python scripts/bench_rollout.py || exit 1
for m in ai league; do
  timeout -k 10 400 python bench.py --mode $m --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_$m.json 2> gpurun_out/b_$m.err || { echo "bench $m failed"; tail -20 gpurun_out/b_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_$m.json')); print('$m', d['value']/1e6, 'M', d['ms_per_step'], 'ms/step')"
done
