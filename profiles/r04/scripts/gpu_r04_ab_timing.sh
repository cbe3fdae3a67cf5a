#!/bin/bash
# A/B: cost of the HIP-event pair around each timed rollout launch (bench --timing-every 1 / 4 / 0), config 2 and
# the league leg, three alternating repeats each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for te in ${TES:-1 4 0}; do
    for m in ${MODES:-ai}; do
      timeout -k 10 200 python bench.py --mode $m --steps 30 --warmup 5 --no-cpu-baseline --timing-every $te \
          > gpurun_out/ab/${m}_te${te}_$rep.json 2> gpurun_out/ab/${m}_te${te}_$rep.err || { tail -20 gpurun_out/ab/${m}_te${te}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/ab/${m}_te${te}_$rep.json')); print('$m te=$te rep=$rep', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['roofline']['avg_kernel_ms'])"
    done
  done
done
