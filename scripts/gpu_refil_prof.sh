#!/bin/bash
# REFIL: the config-5 learner parity test, then bench --mode refil plain and under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_refil_learner.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/refil_learner_tests.log 2>&1 || { tail -30 gpurun_out/refil_learner_tests.log; exit 1; }
tail -2 gpurun_out/refil_learner_tests.log
timeout -k 10 300 python bench.py --mode refil --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_refil.json 2> gpurun_out/bench_refil.err \
    || { echo "bench refil failed"; tail -20 gpurun_out/bench_refil.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_refil.json')); print('refil', d['value']/1e6, 'M', d['ms_per_step'], 'ms/step', 'rollout', d['roofline']['avg_kernel_ms'], 'frac', d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_refil" -o run \
    -- python bench.py --mode refil --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_refil.json 2> gpurun_out/prof_refil.err \
    || { echo "rocprof refil failed"; tail -20 gpurun_out/prof_refil.err; exit 1; }
python scripts/prof_top.py gpurun_out/prof_refil/run_kernel_stats.csv 16
