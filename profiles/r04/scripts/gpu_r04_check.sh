#!/bin/bash
# Round-4 check: new full-shape parity tests, the whole GPU suite + smoke, the default bench (config 2 + league +
# REFIL legs + CPU baselines), and the self-launched 2-rank bench rehearsed with gloo on the box's one GPU.
# Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
if [ -n "$NEW_ONLY" ]; then
  timeout -k 10 400 $T tests/test_gpu_rollout.py::test_rollout_headline_config_agent_parity \
      tests/test_gpu_rollout.py::test_stepper_summary_ring_runahead_matches_resolved \
      tests/test_gpu_refil.py::test_rollout_config5_full_shape tests/test_gpu_refil.py::test_rollout_full_write_slot_extents \
      tests/test_gpu_rollout.py::test_rollout_ring_mode_zero_copy_insert tests/test_gpu_selfplay.py::test_selfplay_ring_mode_equals_plain \
      > gpurun_out/tests_new.log 2>&1 \
      || { tail -40 gpurun_out/tests_new.log; exit 1; }
  tail -2 gpurun_out/tests_new.log
fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 $T tests -m gpu > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
  tail -2 gpurun_out/tests.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 \
      || { tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json')); L=d['league']; R=d['refil']
print('ai', round(d['value']/1e6,2), round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3),
      '| league', round(L['value']/1e6,2), round(L['ms_per_step'],3), '| refil', round(R['value']/1e6,2), round(R['ms_per_step'],3),
      'frac', round(R['roofline_frac'],3), '| cpu', [round(x['value']) for x in d['cpu_baseline']['legs']], R['cpu_baseline']['value'])"
if [ -z "$SKIP_REHEARSAL" ]; then
  timeout -k 10 300 python bench.py --gpus 2 --backend gloo --device 0 --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo "2-rank rehearsal failed"; tail -30 gpurun_out/bench_gloo2.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/bench_gloo2.json')); L=d['league']
print('gloo2 n_gpus', d['n_gpus'], 'ai', round(d['value']/1e6,2), '| league', round(L['value']/1e6,2), L['world_size'], L['collective_backend'], L['league_iterations'], '| refil', round(d['refil']['value']/1e6,2))"
fi
