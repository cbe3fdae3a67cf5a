#!/bin/bash
# Self-play kernel check on the GPU box: the self-play GPU tests, a league-mode bench, and the sp stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_selfplay.py -x -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/sp_tests.log 2>&1 || { tail -30 gpurun_out/sp_tests.log; exit 1; }
tail -2 gpurun_out/sp_tests.log
timeout -k 10 300 python bench.py --mode league --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sp_bench.json \
    2> gpurun_out/sp_bench.err || { echo "bench failed"; tail -20 gpurun_out/sp_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sp_bench.json')); print('league', d['value']/1e6, 'M env-steps/s', d['ms_per_step'], 'ms/step', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'])"
MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 300 python scripts/stamps_sp.py \
    > gpurun_out/stamps_sp.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps_sp.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_sp.txt | head -30
