#!/bin/bash
# bench legs with the rollout's timing end event reused as the run-summary event (default) vs an event of its own
# (MLG_AB_OWN_EVENT=1: an A/B switch in ParallelStepper._queue_summary, removed after the run), alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/event_ab
for rep in 1 2 3; do
  for v in reuse own; do
    if [ $v = own ]; then export MLG_AB_OWN_EVENT=1; else unset MLG_AB_OWN_EVENT; fi
    for m in ai league; do
      timeout -k 10 300 python bench.py --mode $m --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/event_ab/${m}_${v}_$rep.json \
        2> gpurun_out/event_ab/${m}_${v}_$rep.err || { echo "bench $m $v failed"; tail -5 gpurun_out/event_ab/${m}_${v}_$rep.err; exit 1; }
    done
    python3 -c "
import json; a=json.load(open('gpurun_out/event_ab/ai_${v}_$rep.json')); l=json.load(open('gpurun_out/event_ab/league_${v}_$rep.json'))
print('$v $rep ai', round(a['value']/1e6,2), round(a['ms_per_step'],4), 'kern', round(a['roofline']['avg_kernel_ms'],4), '| league', round(l['value']/1e6,2), round(l['ms_per_step'],4), 'kern', round(l['avg_kernel_ms'],4))"
  done
done
