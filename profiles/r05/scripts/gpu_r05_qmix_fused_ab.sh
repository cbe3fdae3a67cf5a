#!/bin/bash
# QMIX learner: fc2 + mixer weight gradients as extra workgroups of the reverse-recurrence launch (default) vs on a
# side stream with events (variant library `side`): learner microbenchmark + the bench's config-2 and league legs.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fused_ab
for rep in 1 2 3; do
  for v in fused side; do
    lib=""; [ $v = side ] && lib=ma-league_amd/maleague/_lib/variants/side.so
    MLG_LIB=$lib MODE=qmix timeout -k 10 200 python scripts/bench_learner.py > gpurun_out/fused_ab/lrn_${v}_$rep.json 2>/dev/null \
      || { echo "learner $v failed"; exit 1; }
    for m in ai league; do
      MLG_LIB=$lib timeout -k 10 300 python bench.py --mode $m --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/fused_ab/${m}_${v}_$rep.json 2> gpurun_out/fused_ab/${m}_${v}_$rep.err \
        || { echo "bench $m $v failed"; tail -5 gpurun_out/fused_ab/${m}_${v}_$rep.err; exit 1; }
    done
    python3 -c "
import json; l=json.load(open('gpurun_out/fused_ab/lrn_${v}_$rep.json')); a=json.load(open('gpurun_out/fused_ab/ai_${v}_$rep.json')); g=json.load(open('gpurun_out/fused_ab/league_${v}_$rep.json'))
print('$v $rep learner', round(l['train_ms'],4), l['loss'], l['grad_norm'], '| ai', round(a['value']/1e6,2), round(a['ms_per_step'],4), '| league', round(g['value']/1e6,2), round(g['ms_per_step'],4))"
  done
done
