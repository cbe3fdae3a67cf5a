#!/bin/bash
# All GPU tests, REFIL rollout microbenchmark (main lib + variants), config-2 and REFIL bench lines, learner kernel
# times under rocprofv3 (ai mode). Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
for v in main ${VARIANTS:-}; do
  lib=""; [ "$v" != main ] && lib=ma-league_amd/maleague/_lib/variants/$v.so
  MLG_LIB=$lib timeout -k 10 200 python scripts/bench_refil_rollout.py > gpurun_out/roll_$v.txt 2>&1 || { echo "rollout $v failed"; tail -20 gpurun_out/roll_$v.txt; exit 1; }
  echo "$v: $(grep -v amdgpu.ids gpurun_out/roll_$v.txt | tail -1)"
done
for m in ai refil; do
  timeout -k 10 300 python bench.py --mode $m --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err \
      || { echo "bench $m failed"; tail -20 gpurun_out/bench_$m.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$m.json')); print('$m', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['avg_kernel_ms'],4))"
done
export TMPDIR=/tmp
for m in ${PROF:-ai refil}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$m" -o run \
      -- python bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$m.json 2> gpurun_out/prof_$m.err \
      || { echo "rocprof $m failed"; tail -20 gpurun_out/prof_$m.err; exit 1; }
  python scripts/prof_top.py gpurun_out/prof_$m/run_kernel_stats.csv 10
done
