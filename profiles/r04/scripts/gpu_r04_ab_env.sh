#!/bin/bash
# A/B of an environment switch of the default library on a rollout microbenchmark: BENCH (default
# scripts/bench_refil_rollout.py) run REPS times alternating with and without ENVSET (e.g. MLG_REFIL_GENERIC=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/abenv
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
  for v in def alt; do
    if [ $v = alt ]; then e="env ${ENVSET}"; else e=""; fi
    $e timeout -k 10 200 python ${BENCH:-scripts/bench_refil_rollout.py} > $O/${v}_$rep.txt 2>&1 \
        || { echo "$v failed"; tail -20 $O/${v}_$rep.txt; exit 1; }
    echo "$v $rep: $(tail -1 $O/${v}_$rep.txt)"
  done
done
