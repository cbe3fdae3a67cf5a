#!/bin/bash
# REFIL dev loop: REFIL tests (rollout + learner), rollout microbench, bench --mode refil, phase stamps.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_refil.py tests/test_gpu_refil_learner.py -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/refil_tests.log 2>&1
rc=$?
tail -3 gpurun_out/refil_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/refil_tests.log; exit 1; }
timeout -k 10 200 python scripts/bench_refil_rollout.py || exit 1
timeout -k 10 400 python bench.py --mode refil --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_refil.json 2> gpurun_out/bench_refil.err || { tail -20 gpurun_out/bench_refil.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_refil.json')); print('bench refil', d['value']/1e6, 'M env-steps/s', d['ms_per_step'], 'ms/step', 'rollout', d['roofline']['avg_kernel_ms'], 'ms')"
if [ -n "$STAMPS" ]; then MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 200 python scripts/stamps_refil.py; fi
