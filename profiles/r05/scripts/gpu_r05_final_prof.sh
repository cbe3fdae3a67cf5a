#!/bin/bash
# The default bench command under rocprofv3 --kernel-trace --stats (the contract's "same command"): its JSON line and
# the per-kernel summary, whose rollout averages must agree with the line's HIP-event avg_kernel_ms.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/final_prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/final_prof/trace" -o run \
    -- python3 bench.py > gpurun_out/final_prof/bench.json 2> gpurun_out/final_prof/bench.err \
    || { echo "profiled bench failed"; tail -20 gpurun_out/final_prof/bench.err; exit 1; }
python3 - <<'PY'
import csv, json
d = json.load(open("gpurun_out/final_prof/bench.json"))
rows = {r["Name"]: r for r in csv.DictReader(open("gpurun_out/final_prof/trace/run_kernel_stats.csv"))}
def avg(key):
    for n, r in rows.items():
        if key in n:
            return float(r["AverageNs"]) / 1e6, int(r["Calls"])
    return None, 0
print("ai", round(d["value"] / 1e6, 2), "hip-event kernel ms", round(d["roofline"]["avg_kernel_ms"], 4),
      "rocprof", avg("rollout_v2_kernel<64, true, 5, 10>"))
L, R = d["league"], d["refil"]
print("league", round(L["value"] / 1e6, 2), "hip-event", round(L["avg_kernel_ms"], 4), "rocprof", avg("rollout_sp8_kernel<10, 10>"))
print("refil", round(R["value"] / 1e6, 2), "hip-event", round(R["avg_kernel_ms"], 4), "rocprof", avg("refil_rollout4_kernel<2, 16>"))
PY
