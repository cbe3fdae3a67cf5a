#!/bin/bash
# Learner GPU tests (split mixer default), then the full bench with the split mixer and with MLG_MIX_FUSED=1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner.py tests/test_checkpoint.py tests/test_gpu_selfplay.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_mix.log 2>&1 || { tail -40 gpurun_out/tests_mix.log; exit 1; }
tail -1 gpurun_out/tests_mix.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mode ai > gpurun_out/bench_split_$rep.json 2> gpurun_out/bench_split.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_split.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_split_$rep.json'));print('split', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_kernel_ms'])"
MLG_MIX_FUSED=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mode ai > gpurun_out/bench_fused_$rep.json 2> gpurun_out/bench_fused.err || { echo "bench fused failed rc=$?"; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_fused_$rep.json'));print('fused', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_kernel_ms'])"
done
export TMPDIR=/tmp
rm -rf gpurun_out/prof_mix
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mix -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --mode ai > gpurun_out/prof_mix.json 2> gpurun_out/prof_mix.err || { echo "rocprof failed"; exit 1; }
f=$(ls gpurun_out/prof_mix/*/run_kernel_stats.csv gpurun_out/prof_mix/run_kernel_stats.csv 2>/dev/null | head -1)
python scripts/prof_top.py "$f" 14
