#!/bin/bash
# REFIL learner change check: its GPU tests, then train() A/B (this tree vs the PRE variant library, 2 repetitions,
# scripts/bench_learner.py MODE=refil) and a rocprofv3 kernel split of this tree's train() calls.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/lrn2
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T ${TESTS:-tests/test_gpu_refil_learner.py} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PRE=${PRE:-prelrn}
for rep in 1 2; do
  for v in def $PRE; do
    lib=ma-league_amd/maleague/_lib/libmaleague.so
    [ $v = def ] || lib=ma-league_amd/maleague/_lib/variants/$v.so
    MODE=${MODE:-refil} MLG_LIB=$lib timeout -k 10 300 python scripts/bench_learner.py > $O/${v}_$rep.json 2> $O/${v}_$rep.err \
        || { echo "bench $v failed"; tail -20 $O/${v}_$rep.err; exit 1; }
    echo "$v $rep $(cat $O/${v}_$rep.json)"
  done
done
MODE=${MODE:-refil} REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python scripts/bench_learner.py > $O/prof.json 2> $O/prof.err || { echo "prof failed"; tail -20 $O/prof.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["AverageNs"])/1e3:8.1f} us x{r["Calls"]:>4}  {r["Name"][:70]}')
PY
