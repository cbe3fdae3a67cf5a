#!/bin/bash
# Learner microbenchmark (scripts/bench_learner.py) under rocprofv3 --kernel-trace --stats for each setting in SETTINGS
# ("name:ENV=VAL,ENV2=VAL2" ...; "base:" = no extra environment); prints per-kernel averages and the last call's timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/lrn_prof
for s in ${SETTINGS:-base:}; do
  name=${s%%:*}; envs=${s#*:}
  ( IFS=,; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    MODE=${MODE:-refil} REPS=${REPS:-20} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$GRAFT_REPO_ROOT/gpurun_out/lrn_prof/$name" -o run -- python3 scripts/bench_learner.py \
      > gpurun_out/lrn_prof/$name.json 2> gpurun_out/lrn_prof/$name.err ) \
    || { echo "setting $name failed"; tail -20 gpurun_out/lrn_prof/$name.err; exit 1; }
  echo "== $name $(cat gpurun_out/lrn_prof/$name.json)"
  python3 - "$GRAFT_REPO_ROOT/gpurun_out/lrn_prof/$name/run_kernel_stats.csv" "$GRAFT_REPO_ROOT/gpurun_out/lrn_prof/$name/run_kernel_trace.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'  {float(r["AverageNs"])/1e3:9.1f} us x{int(r["Calls"]):4d}  {r["Name"].replace("(anonymous namespace)::", "")[:60]}')
tr = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[2])))
starts = [i for i, r in enumerate(tr) if "prologue_kernel" in r[2] or "prep_kernel" in r[2]]
if len(starts) >= 2:
    a, b = starts[-2], starts[-1]
    t0 = tr[a][0]
    print("  last call timeline (start us, dur us):")
    for s_, e_, n_ in tr[a:b]:
        print(f'    {(s_ - t0) / 1e3:8.1f} {(e_ - s_) / 1e3:7.1f}  {n_.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:50]}')
PY
done
