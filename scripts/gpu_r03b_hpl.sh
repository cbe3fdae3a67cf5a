#!/bin/bash
# v7 h planes + split mixer: rollout / episode / learner GPU tests, fixed-policy rollout timing, learner
# microbenchmark (split mixer vs MLG_MIX_FUSED=1) under a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py::test_rollout_v7_split_bf16_gru_matches_fp32 tests/test_gpu_rollout.py tests/test_gpu_episode.py tests/test_gpu_learner.py tests/test_checkpoint.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_hpl.log 2>&1 || { tail -40 gpurun_out/tests_hpl.log; exit 1; }
tail -1 gpurun_out/tests_hpl.log
for rep in 1 2; do
  RING=1 timeout -k 10 200 python scripts/bench_rollout.py > gpurun_out/ro_hpl_$rep.json 2>/dev/null || { echo "bench failed"; exit 1; }
  cat gpurun_out/ro_hpl_$rep.json
done
run() {  # name env
  rm -rf gpurun_out/lprof_$1
  env $2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof_$1 -o run -- python scripts/bench_learner.py > gpurun_out/lb_$1.json 2> gpurun_out/lb_$1.err || { echo "$1 failed"; tail -5 gpurun_out/lb_$1.err; return 1; }
  echo "== $1 $(cat gpurun_out/lb_$1.json)"
  f=$(ls gpurun_out/lprof_$1/*/run_kernel_stats.csv gpurun_out/lprof_$1/run_kernel_stats.csv 2>/dev/null | head -1)
  python scripts/prof_top.py "$f" 14 | grep -v rollout
}
run split MLG_X=0 || exit 1
run fused MLG_MIX_FUSED=1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python scripts/bench_learner.py > gpurun_out/lbs_$rep.json 2>/dev/null && echo "split: $(cat gpurun_out/lbs_$rep.json)"
  MLG_MIX_FUSED=1 timeout -k 10 200 python scripts/bench_learner.py > gpurun_out/lbf_$rep.json 2>/dev/null && echo "fused: $(cat gpurun_out/lbf_$rep.json)"
done
