#!/bin/bash
# Dev GPU session: GPU tests, bench, stamps of both rollout kernels. Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?
tail -5 gpurun_out/tests.log
[ $rc -eq 0 ] || { echo "tests failed rc=$rc"; exit 1; }
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; exit 1; }
cat gpurun_out/bench.json
for k in v1 v2; do
  MLG_ROLLOUT_KERNEL=$k MLG_LIB=ma-league_amd/maleague/_lib/libmaleague_stamps.so timeout -k 10 300 python scripts/stamps_rollout.py > gpurun_out/stamps_$k.txt 2>&1 || { echo "stamps $k failed"; exit 1; }
  echo "== $k"; cat gpurun_out/stamps_$k.txt
done
