#!/bin/bash
# REFIL path check: REFIL GPU tests, refil bench line, REFIL phase stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_refil.py tests/test_gpu_refil_learner.py -x -q --timeout 150 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/rq_tests.log 2>&1 || { tail -30 gpurun_out/rq_tests.log; exit 1; }
tail -1 gpurun_out/rq_tests.log
timeout -k 10 300 python bench.py --mode refil --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rq_bench.json \
    2> gpurun_out/rq_bench.err || { echo "bench failed"; tail -20 gpurun_out/rq_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/rq_bench.json')); print('refil', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],3), 'ms/step', d['roofline']['kernel'], round(d['roofline']['avg_kernel_ms'],4))"
MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 300 python scripts/stamps_refil.py \
    > gpurun_out/stamps_refil.txt 2>&1 || { echo "stamps failed"; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_refil.txt | tail -10
