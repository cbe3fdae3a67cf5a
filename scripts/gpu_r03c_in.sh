#!/bin/bash
# agent_in timestep-loop A/B: learner GPU tests on the default build, then per variant (MLG_IN_TS) the learner
# kernel times under a kernel trace and a config-2 bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_learner.py tests/test_checkpoint.py tests/test_gpu_episode.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_in.log 2>&1 || { tail -40 gpurun_out/tests_in.log; exit 1; }
tail -1 gpurun_out/tests_in.log
for v in default ts1 ts2 ts8; do
  lib=""; [ "$v" != default ] && lib="$GRAFT_REPO_ROOT/ma-league_amd/maleague/_lib/variants/$v.so"
  rm -rf gpurun_out/inprof_$v
  MLG_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/inprof_$v -o run -- python scripts/bench_learner.py > gpurun_out/in_lb_$v.json 2> gpurun_out/in_lb_$v.err || { echo "lb $v failed"; tail -5 gpurun_out/in_lb_$v.err; exit 1; }
  f=$(ls gpurun_out/inprof_$v/*/run_kernel_stats.csv gpurun_out/inprof_$v/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "== $v"; python scripts/prof_top.py "$f" 14 | grep -v rollout | grep -i "agent_in\|bwd4\|rec4"
done
for v in default ts1 ts2; do
  lib=""; [ "$v" != default ] && lib="$GRAFT_REPO_ROOT/ma-league_amd/maleague/_lib/variants/$v.so"
  MLG_LIB=$lib timeout -k 10 300 python bench.py --mode ai --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/in_b_$v.json 2> gpurun_out/in_b_$v.err || { echo "bench $v failed"; tail -20 gpurun_out/in_b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/in_b_$v.json')); print('$v', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), 'ms/step')"
done
