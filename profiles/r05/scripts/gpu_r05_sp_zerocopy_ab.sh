#!/bin/bash
# League leg: self-play run summaries zero-copy (pinned slot read by record_runs, default) vs device buffer + D2H copy
# + event (MLG_AB_SP_DEVCOPY=1: an A/B switch in SelfPlayParallelStepper, removed after the run), alternating;
# first the self-play / league GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/spzc_ab
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_selfplay.py -m gpu \
  > gpurun_out/spzc_ab/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/spzc_ab/tests.log; exit 1; }
tail -1 gpurun_out/spzc_ab/tests.log
for rep in 1 2 3; do
  for v in zc dev; do
    if [ $v = dev ]; then export MLG_AB_SP_DEVCOPY=1; else unset MLG_AB_SP_DEVCOPY; fi
    timeout -k 10 300 python bench.py --mode league --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/spzc_ab/league_${v}_$rep.json \
      2> gpurun_out/spzc_ab/league_${v}_$rep.err || { echo "bench $v failed"; tail -5 gpurun_out/spzc_ab/league_${v}_$rep.err; exit 1; }
    python3 -c "
import json; g=json.load(open('gpurun_out/spzc_ab/league_${v}_$rep.json'))
print('$v $rep league', round(g['value']/1e6,2), round(g['ms_per_step'],4), 'kern', round(g['roofline']['avg_kernel_ms'],4), 'games', g.get('payoff_games'), 'hist', g.get('historical_matches_timed_rank0'))"
  done
done
