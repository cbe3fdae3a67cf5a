#!/bin/bash
# Full bench (config 2 + league legs) with the split mixer and with MLG_MIX_FUSED=1, then a kernel-trace profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_split.json 2> gpurun_out/bench_split.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_split.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_split.json'));print('split', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_kernel_ms'], d['league']['value']/1e6)"
MLG_MIX_FUSED=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_fused.json 2> gpurun_out/bench_fused.err || { echo "bench fused failed rc=$?"; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_fused.json'));print('fused', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_kernel_ms'], d['league']['value']/1e6)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_split2.json 2> /dev/null || { echo "bench failed"; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_split2.json'));print('split', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_kernel_ms'], d['league']['value']/1e6)"
rm -rf gpurun_out/prof_ai
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ai -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --mode ai > gpurun_out/prof_ai.json 2> gpurun_out/prof_ai.err || { echo "rocprof failed"; exit 1; }
f=$(ls gpurun_out/prof_ai/*/run_kernel_stats.csv gpurun_out/prof_ai/run_kernel_stats.csv 2>/dev/null | head -1)
python scripts/prof_top.py "$f" 14
