#!/bin/bash
# Rollout microbenchmark of every variant library under ma-league_amd/maleague/_lib/variants/.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for so in ma-league_amd/maleague/_lib/variants/*.so; do
  n=$(basename $so .so)
  MLG_LIB=$so timeout -k 10 300 python scripts/bench_rollout.py > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || { echo "$n failed"; tail -5 gpurun_out/var_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/var_$n.json)"
done
