#!/bin/bash
# Learner GPU tests + learner microbenchmark under a kernel trace (per-kernel averages).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner.py tests/test_checkpoint.py tests/test_gpu_episode.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_lrn.log 2>&1 || { tail -40 gpurun_out/tests_lrn.log; exit 1; }
tail -1 gpurun_out/tests_lrn.log
rm -rf gpurun_out/lprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof -o run -- python scripts/bench_learner.py > gpurun_out/lb.json 2> gpurun_out/lb.err || { echo "lb failed"; tail -5 gpurun_out/lb.err; exit 1; }
cat gpurun_out/lb.json
f=$(ls gpurun_out/lprof/*/run_kernel_stats.csv gpurun_out/lprof/run_kernel_stats.csv 2>/dev/null | head -1)
python scripts/prof_top.py "$f" 14 | grep -v rollout
