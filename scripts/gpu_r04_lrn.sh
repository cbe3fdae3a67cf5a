#!/bin/bash
# Learner A/B: the learner GPU tests, then the train() microbenchmark (scripts/bench_learner.py) for QMIX and REFIL
# with the default build vs an env switch (AB_ENV, e.g. MLG_REFIL_REC16=1), alternating, and a rocprofv3 stats run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/lrn
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T ${TESTS:-tests/test_gpu_learner.py tests/test_gpu_refil_learner.py} > gpurun_out/lrn/tests.log 2>&1 \
    || { tail -40 gpurun_out/lrn/tests.log; exit 1; }
tail -1 gpurun_out/lrn/tests.log
for rep in 1 2; do
  for mode in ${LMODES:-qmix refil}; do
    MODE=$mode timeout -k 10 200 python scripts/bench_learner.py > gpurun_out/lrn/${mode}_def_$rep.json 2> gpurun_out/lrn/err.txt \
        || { tail -20 gpurun_out/lrn/err.txt; exit 1; }
    echo "$mode default $(cat gpurun_out/lrn/${mode}_def_$rep.json)"
    if [ -n "$AB_ENV" ]; then
      env $AB_ENV MODE=$mode timeout -k 10 200 python scripts/bench_learner.py > gpurun_out/lrn/${mode}_ab_$rep.json 2> gpurun_out/lrn/err.txt \
          || { tail -20 gpurun_out/lrn/err.txt; exit 1; }
      echo "$mode $AB_ENV $(cat gpurun_out/lrn/${mode}_ab_$rep.json)"
    fi
  done
done
for mode in ${LMODES:-qmix refil}; do
  MODE=$mode REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/lrn/prof_$mode" -o run \
      -- python3 scripts/bench_learner.py > gpurun_out/lrn/prof_$mode.json 2> gpurun_out/lrn/err.txt || { tail -20 gpurun_out/lrn/err.txt; exit 1; }
  python3 scripts/prof_top.py gpurun_out/lrn/prof_$mode/run_kernel_stats.csv 14
done
