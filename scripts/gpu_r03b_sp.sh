#!/bin/bash
# sp7 h planes: self-play + league GPU tests, then the league bench leg twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_rollout.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests_sp.log 2>&1 || { tail -40 gpurun_out/tests_sp.log; exit 1; }
tail -1 gpurun_out/tests_sp.log
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --mode league > gpurun_out/bench_league_$rep.json 2> gpurun_out/bench_league.err || { echo "bench failed rc=$?"; tail -5 gpurun_out/bench_league.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/bench_league_$rep.json'));l=d.get('league',d)
print('league', l['value']/1e6, l['ms_per_step'], l.get('avg_kernel_ms'), l.get('roofline_frac'))"
done
