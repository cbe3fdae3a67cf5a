#!/bin/bash
# rollout GPU tests, then fixed-policy rollout timing: default library and each variant, 3 alternating reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_episode.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_ab.log 2>&1 || { tail -40 gpurun_out/tests_ab.log; exit 1; }
tail -1 gpurun_out/tests_ab.log
for rep in 1 2 3; do
  RING=1 timeout -k 10 200 python scripts/bench_rollout.py > gpurun_out/ab_default_$rep.json 2>/dev/null || { echo "bench default failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_default_$rep.json'))['v7'];print('default', round(d['kernel_ms'],4), round(d['min_ms'],4))"
  for v in $VARIANTS; do
    MLG_LIB=ma-league_amd/maleague/_lib/variants/$v.so RING=1 timeout -k 10 200 python scripts/bench_rollout.py > gpurun_out/ab_${v}_$rep.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${v}_$rep.json'))['v7'];print('$v', round(d['kernel_ms'],4), round(d['min_ms'],4))"
  done
done
