#!/bin/bash
# A/B of variant libraries on a fixed-policy rollout microbenchmark: BENCH (default scripts/bench_refil_rollout.py),
# VARIANTS (names under _lib/variants/, "def" = the default library), REPS alternating repetitions.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-def}; do
    lib=ma-league_amd/maleague/_lib/libmaleague.so
    [ $v = def ] || lib=ma-league_amd/maleague/_lib/variants/$v.so
    MLG_LIB=$lib timeout -k 10 200 python ${BENCH:-scripts/bench_refil_rollout.py} > $O/${v}_$rep.txt 2>&1 \
        || { echo "$v failed"; tail -20 $O/${v}_$rep.txt; exit 1; }
    echo "$v $rep: $(tail -1 $O/${v}_$rep.txt)"
  done
done
