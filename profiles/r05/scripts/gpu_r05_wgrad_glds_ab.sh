#!/bin/bash
# Blocked wgrad with the next step's rows staged global -> LDS (default) vs variant libraries in VARIANTS
# (maleague/_lib/variants/<name>.so; `noglds` = -DMLG_WGRAD_NOGLDS, register loads with no prefetch; `head` = the
# previous commit): learner GPU tests, then learner microbenchmarks (REFIL, QMIX) and the bench's config-2 and REFIL
# legs, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/glds_ab
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 $T tests -m gpu -k "learner or wgrad or refil" > gpurun_out/glds_ab/tests.log 2>&1 \
    || { tail -30 gpurun_out/glds_ab/tests.log; exit 1; }
  tail -1 gpurun_out/glds_ab/tests.log
fi
for rep in ${ROUNDS:-1 2}; do
  for v in glds ${VARIANTS:-noglds}; do
    lib=""; [ $v != glds ] && lib=ma-league_amd/maleague/_lib/variants/$v.so
    for lm in ${LRN_MODES:-refil qmix}; do
      MLG_LIB=$lib MODE=$lm timeout -k 10 200 python scripts/bench_learner.py > gpurun_out/glds_ab/lrn_${lm}_${v}_$rep.json 2> gpurun_out/glds_ab/lrn_${lm}_${v}_$rep.err \
        || { echo "learner $lm $v failed"; tail -15 gpurun_out/glds_ab/lrn_${lm}_${v}_$rep.err; exit 1; }
    done
    for m in ${BENCH_MODES:-ai refil}; do
      MLG_LIB=$lib timeout -k 10 300 python bench.py --mode $m --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/glds_ab/${m}_${v}_$rep.json 2> gpurun_out/glds_ab/${m}_${v}_$rep.err \
        || { echo "bench $m $v failed"; tail -5 gpurun_out/glds_ab/${m}_${v}_$rep.err; exit 1; }
    done
    python3 - "$v" "$rep" <<'PY'
import json, os, sys
v, rep = sys.argv[1], sys.argv[2]
d = "gpurun_out/glds_ab/"
out = [v, rep]
for lm in ("refil", "qmix"):
    f = d + f"lrn_{lm}_{v}_{rep}.json"
    if os.path.exists(f):
        l = json.load(open(f))
        out += [f"{lm}-lrn", round(l["train_ms"], 4), l["loss"]]
for m in ("ai", "refil"):
    f = d + f"{m}_{v}_{rep}.json"
    if os.path.exists(f):
        out += [m, round(json.load(open(f))["value"] / 1e6, 2)]
print(*out)
PY
  done
done
