#!/bin/bash
# Round 6: counters of the self-play kernels at HEAD (sp8 on the bench's composed-team league leg; sp7 forced with
# MLG_ROLLOUT_KERNEL=sp7), merged into a copy of profiles/counters.json, then the default `python3 bench.py` under
# rocprofv3 --kernel-trace --stats (the driver's command).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
MODES=league COMMIT=${COMMIT:-unknown} bash scripts/gpu_counters.sh > gpurun_out/cnt_sp8.log 2>&1 || { tail -20 gpurun_out/cnt_sp8.log; exit 1; }
cp gpurun_out/counters/counters.json gpurun_out/counters_sp8.json
mv gpurun_out/counters gpurun_out/counters_sp8_raw
MLG_ROLLOUT_KERNEL=sp7 MODES=league COMMIT=${COMMIT:-unknown} MERGE=gpurun_out/counters_sp8.json bash scripts/gpu_counters.sh \
    > gpurun_out/cnt_sp7.log 2>&1 || { tail -20 gpurun_out/cnt_sp7.log; exit 1; }
cp gpurun_out/counters/counters.json gpurun_out/counters_sp8_sp7.json
python3 -c "
import json; d=json.load(open('gpurun_out/counters_sp8_sp7.json'))['kernels']
for k in ('rollout_sp8_kernel<10, 10>', 'rollout_sp7_kernel<10, 10>'):
    v=d.get(k, {}); print(k, {x: v.get(x) for x in ('commit','hbm_bytes_per_launch','mfma_busy','wait_any_frac','valu_per_mfma')})"
mkdir -p gpurun_out/final_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/final_prof" -o run \
    -- python3 bench.py > gpurun_out/final_prof/bench.json 2> gpurun_out/final_prof/bench.err || { tail -20 gpurun_out/final_prof/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/final_prof/bench.json')); print('final', round(d['value']/1e6,2), d['roofline']['avg_kernel_ms'], d['league']['value']/1e6, d['refil']['value']/1e6)"
