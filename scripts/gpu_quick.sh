#!/bin/bash
# Quick GPU step: the whole GPU suite (or TESTS=...), then the default bench line and (TRACE=1) the
# per-iteration timelines of MODES under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q ${PYTEST_ARGS:-} --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 $T ${TESTS:-tests -m gpu} > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
  tail -3 gpurun_out/smoke.log
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err \
      || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench.json')); L=d.get('league'); R=d.get('refil')
print('ai', round(d['value']/1e6,2), round(d['ms_per_step'],4), 'kern', round(d['roofline']['avg_kernel_ms'],4), 'frac', round(d['roofline']['frac'],3))
if L: print('league', round(L['value']/1e6,2), round(L['ms_per_step'],4), 'kern', round(L['avg_kernel_ms'],4), 'exch', round(L['exchange_ms_mean'],3))
if R: print('refil', round(R['value']/1e6,2), round(R['ms_per_step'],4), 'kern', round(R['avg_kernel_ms'],4), 'len', round(R['mean_episode_len'],2))"
fi
if [ -n "$TRACE" ]; then
  for m in ${MODES:-ai league refil}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/trace_$m" -o run \
        -- python3 bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace_$m.json 2> gpurun_out/trace_$m.err \
        || { echo "trace $m failed"; tail -20 gpurun_out/trace_$m.err; exit 1; }
    key=$( [ $m = ai ] && echo rollout_v2_kernel || ( [ $m = league ] && echo rollout_sp || echo refil_rollout ) )
    python3 scripts/trace_iter.py gpurun_out/trace_$m/run_kernel_trace.csv $key 6 > gpurun_out/trace_$m.txt || exit 1
    head -${TRACE_LINES:-24} gpurun_out/trace_$m.txt
  done
fi
