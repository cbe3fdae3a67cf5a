#!/bin/bash
# Blocked wgrad with the next step's rows staged global -> LDS (default) vs variant libraries in VARIANTS
# (maleague/_lib/variants/<name>.so; `noglds` = -DMLG_WGRAD_NOGLDS, register loads with no prefetch; `head` = the
# previous commit): learner GPU tests, then learner microbenchmarks (REFIL, QMIX) and the bench's config-2 and REFIL
# legs, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/glds_ab
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests -m gpu -k "learner or wgrad or refil" > gpurun_out/glds_ab/tests.log 2>&1 \
  || { tail -30 gpurun_out/glds_ab/tests.log; exit 1; }
tail -1 gpurun_out/glds_ab/tests.log
for rep in ${REPS:-1 2}; do
  for v in glds ${VARIANTS:-noglds}; do
    lib=""; [ $v != glds ] && lib=ma-league_amd/maleague/_lib/variants/$v.so
    for lm in refil qmix; do
      MLG_LIB=$lib MODE=$lm timeout -k 10 200 python scripts/bench_learner.py > gpurun_out/glds_ab/lrn_${lm}_${v}_$rep.json 2>/dev/null \
        || { echo "learner $lm $v failed"; exit 1; }
    done
    for m in ai refil; do
      MLG_LIB=$lib timeout -k 10 300 python bench.py --mode $m --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/glds_ab/${m}_${v}_$rep.json 2> gpurun_out/glds_ab/${m}_${v}_$rep.err \
        || { echo "bench $m $v failed"; tail -5 gpurun_out/glds_ab/${m}_${v}_$rep.err; exit 1; }
    done
    python3 -c "
import json; d='gpurun_out/glds_ab/'
lr=json.load(open(d+'lrn_refil_${v}_$rep.json')); lq=json.load(open(d+'lrn_qmix_${v}_$rep.json'))
a=json.load(open(d+'ai_${v}_$rep.json')); r=json.load(open(d+'refil_${v}_$rep.json'))
print('$v $rep refil-lrn', round(lr['train_ms'],4), lr['loss'], '| qmix-lrn', round(lq['train_ms'],4), lq['loss'], '| ai', round(a['value']/1e6,2), '| refil', round(r['value']/1e6,2))"
  done
done
