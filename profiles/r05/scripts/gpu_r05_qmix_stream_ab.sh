#!/bin/bash
# QMIX learner on one stream vs the fc2 + mixer weight gradients on a side stream: learner microbenchmark (no profiler) and the
# bench's config-2 leg, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/stream_ab_q
for rep in 1 2 3; do
  for v in two one; do
    if [ $v = one ]; then export MLG_LEARNER_ONE_STREAM=1; else unset MLG_LEARNER_ONE_STREAM; fi
    MODE=qmix timeout -k 10 200 python scripts/bench_learner.py > gpurun_out/stream_ab_q/lrn_${v}_$rep.json 2>/dev/null \
      || { echo "learner $v failed"; exit 1; }
    timeout -k 10 300 python bench.py --mode ai --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/stream_ab_q/bench_${v}_$rep.json \
      2> gpurun_out/stream_ab_q/bench_${v}_$rep.err || { echo "bench $v failed"; tail -5 gpurun_out/stream_ab_q/bench_${v}_$rep.err; exit 1; }
    python3 -c "
import json; l=json.load(open('gpurun_out/stream_ab_q/lrn_${v}_$rep.json')); b=json.load(open('gpurun_out/stream_ab_q/bench_${v}_$rep.json'))
print('$v $rep learner', round(l['train_ms'],4), 'loss', l['loss'], '| bench', round(b['value']/1e6,2), round(b['ms_per_step'],4), 'len', round(b.get('mean_episode_len',0),2))"
  done
done
