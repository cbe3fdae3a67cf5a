#!/bin/bash
# Full GPU test suite, REFIL bench (config 5) and its rocprofv3 kernel-trace summary. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?
tail -5 gpurun_out/tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; tail -60 gpurun_out/tests.log; exit 1; }
STEPS=${STEPS:-10}
timeout -k 10 600 python bench.py --mode refil --steps "$STEPS" --warmup 3 > gpurun_out/bench_refil.json 2> gpurun_out/bench_refil.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench_refil.err; exit 1; }
cat gpurun_out/bench_refil.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_refil" -o run -- python bench.py --mode refil --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_refil_bench.json 2> gpurun_out/prof_refil.err || { echo "rocprof failed rc=$?"; tail -20 gpurun_out/prof_refil.err; exit 1; }
cat gpurun_out/prof_refil_bench.json
