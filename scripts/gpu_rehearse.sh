#!/bin/bash
# Multi-rank rehearsal on the 1-GPU box: bench.py --gpus N self-launches N ranks (torch.distributed.run child) with
# gloo collectives and every rank on GPU 0 -- the driver's N-GPU path (league config 3 at N = 2, config 4 with
# AlphaStar roles at N = 4) end to end, minus RCCL.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/rehearse
for n in ${NS:-2 4}; do
  timeout -k 10 600 python bench.py --gpus $n --backend gloo --device 0 --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
      > gpurun_out/rehearse/bench_gloo$n.json 2> gpurun_out/rehearse/bench_gloo$n.err \
      || { echo "rehearsal N=$n failed"; tail -40 gpurun_out/rehearse/bench_gloo$n.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/rehearse/bench_gloo$n.json')); L=d['league']; R=d['refil']
print('N=$n n_gpus', d['n_gpus'], 'ai', round(d['value']/1e6,2), d['config']['parallelism'], '| league', round(L['value']/1e6,2), L['represents'][:40], L['world_size'], L['collective_backend'], 'iters', L['league_iterations'], 'hist', L['historical_snapshots'], 'hist_timed0', L.get('historical_matches_timed_rank0'), 'evict', L['evictions'], 'opp0', L['opponents_rank0'], 'teams', L.get('teams'), 'away0', L.get('away_teams_rank0'), '| refil', round(R['value']/1e6,2))"
done
