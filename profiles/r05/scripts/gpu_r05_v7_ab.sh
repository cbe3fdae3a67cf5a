#!/bin/bash
# A/B of v7 rollout variants (scripts/bench_rollout.py: fixed policy, same episodes, 4096 envs, train mode into the
# replay ring), one process per library, two passes.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/v7_ab
for pass in $(seq 1 ${PASSES:-2}); do
  for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then lib=""; else lib=ma-league_amd/maleague/_lib/variants/$v.so; fi
    MLG_LIB=$lib RING=1 MLG_BENCH_KERNELS=v7 timeout -k 10 200 python scripts/bench_rollout.py > gpurun_out/v7_ab/${v}_$pass.json 2> gpurun_out/v7_ab/${v}_$pass.err \
      || { echo "variant $v failed"; tail -5 gpurun_out/v7_ab/${v}_$pass.err; exit 1; }
    echo "$v pass $pass: $(python3 -c "import json;d=json.load(open('gpurun_out/v7_ab/${v}_$pass.json'))['v7'];print(round(d['kernel_ms'],4), round(d['min_ms'],4), d['mean_len'])")"
  done
done
