#!/bin/bash
# REFIL A/B check: REFIL GPU tests, the fixed-policy rollout microbenchmark and the refil bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_refil.py tests/test_gpu_refil_learner.py -x -q --timeout 150 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/rq_tests.log 2>&1 || { tail -30 gpurun_out/rq_tests.log; exit 1; }
tail -1 gpurun_out/rq_tests.log
timeout -k 10 200 python scripts/bench_refil_rollout.py > gpurun_out/rq_roll.txt 2>&1 || { echo "rollout bench failed"; tail -20 gpurun_out/rq_roll.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/rq_roll.txt | tail -3
for v in ${VARIANTS:-}; do
  MLG_LIB=ma-league_amd/maleague/_lib/variants/$v.so timeout -k 10 200 python scripts/bench_refil_rollout.py > gpurun_out/rq_roll_$v.txt 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/rq_roll_$v.txt; exit 1; }
  echo "variant $v:"; grep -v amdgpu.ids gpurun_out/rq_roll_$v.txt | tail -2
done
timeout -k 10 300 python bench.py --mode refil --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rq_bench.json \
    2> gpurun_out/rq_bench.err || { echo "bench failed"; tail -20 gpurun_out/rq_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/rq_bench.json')); print('refil', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms/step', d['roofline']['kernel'], round(d['roofline']['avg_kernel_ms'],4))"
