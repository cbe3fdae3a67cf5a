#!/bin/bash
# Rollout tests incl. v6, rollout microbench v2 vs v6, bench ai with v6.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_v6.log 2>&1
rc=$?; tail -3 gpurun_out/tests_v6.log
[ $rc -eq 0 ] || { grep -E "^E |Error|assert|FAIL" gpurun_out/tests_v6.log | head -20; exit 1; }
MLG_BENCH_KERNELS=v2,v6,v2,v6 timeout -k 10 300 python scripts/bench_rollout.py || exit 1
MLG_ROLLOUT_KERNEL=v6 timeout -k 10 400 python bench.py --mode ai --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_v6.json 2> gpurun_out/b_v6.err || { echo "bench failed"; tail -20 gpurun_out/b_v6.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_v6.json')); print('ai v6', d['value']/1e6, 'M', d['ms_per_step'], 'ms/step', d['roofline']['avg_kernel_ms'])"
