#!/bin/bash
# Learner A/B under rocprofv3 (scripts/bench_learner.py): per-kernel averages for each setting in SETTINGS
# ("name:ENV=VAL,ENV2=VAL2" ...; "base:" = no extra environment).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/lrn_ab
for s in ${SETTINGS:-base:}; do
  name=${s%%:*}; envs=${s#*:}
  ( IFS=,; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    MODE=${MODE:-refil} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/lrn_ab/$name" -o run \
      -- python3 scripts/bench_learner.py > gpurun_out/lrn_ab/$name.json 2> gpurun_out/lrn_ab/$name.err ) \
    || { echo "setting $name failed"; tail -20 gpurun_out/lrn_ab/$name.err; exit 1; }
  echo "== $name $(cat gpurun_out/lrn_ab/$name.json)"
  python3 - "$GRAFT_REPO_ROOT/gpurun_out/lrn_ab/$name/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'  {float(r["AverageNs"])/1e3:9.1f} us x{int(r["Calls"]):4d}  {r["Name"][:70]}')
PY
done
