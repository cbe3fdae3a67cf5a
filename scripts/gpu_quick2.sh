#!/bin/bash
# Rollout-path check: rollout + self-play GPU tests, ai + league bench lines, v7 stamps (+ one-env timeline when the
# variant library exists).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_selfplay.py -x -q --timeout 150 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/q_tests.log 2>&1 || { tail -30 gpurun_out/q_tests.log; exit 1; }
tail -1 gpurun_out/q_tests.log
for m in ai league; do
  timeout -k 10 300 python bench.py --mode $m --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/q_bench_$m.json \
      2> gpurun_out/q_bench_$m.err || { echo "bench $m failed"; tail -20 gpurun_out/q_bench_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q_bench_$m.json')); print('$m', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), 'ms/step', d['roofline']['kernel'], round(d['roofline']['avg_kernel_ms'],4))"
done
MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 300 \
    python scripts/stamps_rollout.py > gpurun_out/stamps_v7.txt 2>&1 || { echo "stamps failed"; exit 1; }
grep -E "total cycles|per-WG total|nrun= 1 |nrun=16" gpurun_out/stamps_v7.txt
if [ -f ma-league_amd/maleague/_lib/variants/tl.so ]; then
  TIMELINE=1 MLG_ROLLOUT_KERNEL=v7 MLG_LIB=ma-league_amd/maleague/_lib/variants/tl.so timeout -k 10 300 \
      python scripts/stamps_rollout.py > gpurun_out/stamps_v7_tl.txt 2>&1 || { echo "timeline failed"; exit 1; }
  grep timeline gpurun_out/stamps_v7_tl.txt
fi
