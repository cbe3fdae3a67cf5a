#!/bin/bash
# Zero-copy run summaries: full GPU suite, then config 2 (ai) bench twice and a kernel trace of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_zc.log 2>&1 || { tail -40 gpurun_out/tests_zc.log; exit 1; }
tail -1 gpurun_out/tests_zc.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --mode ai > gpurun_out/bench_zc_$rep.json 2> gpurun_out/bench_zc.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_zc.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_zc_$rep.json'));print('zc', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_kernel_ms'])"
done
export TMPDIR=/tmp
rm -rf gpurun_out/prof_zc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_zc -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --mode ai > gpurun_out/prof_zc.json 2> gpurun_out/prof_zc.err || { echo "rocprof failed"; exit 1; }
f=$(ls gpurun_out/prof_zc/*/run_kernel_stats.csv gpurun_out/prof_zc/run_kernel_stats.csv 2>/dev/null | head -1)
python scripts/prof_top.py "$f" 6
