#!/bin/bash
# A/B of the rollout kernel: rollout GPU tests on the default library, then the fixed-policy microbenchmark
# (ring mode) for the default library and each variant library named in VARIANTS (maleague/_lib/variants/*.so).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_ab.log 2>&1 || { tail -30 gpurun_out/tests_ab.log; exit 1; }
tail -1 gpurun_out/tests_ab.log
for rep in 1 2 3; do
  RING=1 timeout -k 10 200 python scripts/bench_rollout.py > gpurun_out/ab_default_$rep.json 2>/dev/null || { echo "bench default failed"; exit 1; }
  echo "default: $(cat gpurun_out/ab_default_$rep.json)"
  for v in $VARIANTS; do
    MLG_LIB=ma-league_amd/maleague/_lib/variants/$v.so RING=1 timeout -k 10 200 python scripts/bench_rollout.py > gpurun_out/ab_${v}_$rep.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    echo "$v: $(cat gpurun_out/ab_${v}_$rep.json)"
  done
done
