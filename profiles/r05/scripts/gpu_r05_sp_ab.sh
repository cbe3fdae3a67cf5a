#!/bin/bash
# A/B of self-play rollout variants (scripts/bench_sp_rollout.py, one process per library), two passes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sp_ab
for pass in $(seq 1 ${PASSES:-2}); do
  for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then lib=""; else lib=ma-league_amd/maleague/_lib/variants/$v.so; fi
    k=${KERNEL:-}
    MLG_LIB=$lib MLG_ROLLOUT_KERNEL=$k timeout -k 10 200 python scripts/bench_sp_rollout.py > gpurun_out/sp_ab/${v}_$pass.json 2> gpurun_out/sp_ab/${v}_$pass.err \
      || { echo "variant $v failed"; tail -5 gpurun_out/sp_ab/${v}_$pass.err; exit 1; }
    echo "$v pass $pass: $(cat gpurun_out/sp_ab/${v}_$pass.json)"
  done
done
