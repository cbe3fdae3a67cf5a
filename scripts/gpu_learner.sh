#!/bin/bash
# Learner A/B: GPU learner tests, then scripts/bench_learner.py under a kernel-trace profile for the main library
# and every variant under ma-league_amd/maleague/_lib/variants/ (per-kernel averages of the learner kernels).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_learner.py tests/test_checkpoint.py > gpurun_out/learner_tests.log 2>&1 || { tail -30 gpurun_out/learner_tests.log; exit 1; }
tail -1 gpurun_out/learner_tests.log
run() {  # name lib
  rm -rf gpurun_out/lprof_$1
  MLG_LIB=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof_$1 -o run -- python scripts/bench_learner.py > gpurun_out/lb_$1.json 2> gpurun_out/lb_$1.err || { echo "$1 failed"; tail -5 gpurun_out/lb_$1.err; return 1; }
  echo "== $1 $(cat gpurun_out/lb_$1.json)"
  f=$(ls gpurun_out/lprof_$1/*/run_kernel_stats.csv gpurun_out/lprof_$1/run_kernel_stats.csv 2>/dev/null | head -1)
  python scripts/prof_top.py "$f" 16 | grep -v rollout
}
run main ma-league_amd/maleague/_lib/libmaleague.so || exit 1
for so in ma-league_amd/maleague/_lib/variants/*.so; do
  [ -e "$so" ] || continue
  run $(basename $so .so) $so || exit 1
done
