#!/bin/bash
# Alternating A/B of library variants (VARIANTS="name:path/to/lib.so[:ENV=V,ENV2=W] ...", "base:" = the default library,
# "name::ENV=V" = the default library with environment settings) over ROUNDS
# rounds: the learner microbenchmark (LRN_MODES, scripts/bench_learner.py: mean ms per train()) and bench legs
# (BENCH_MODES, bench.py --mode M: value and the rollout kernel's HIP-event average), microbenchmark scripts (SCRIPTS,
# last output line). Optional TESTS run first with
# every variant to check parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
split() { name=${1%%:*}; rest=${1#*:}; lib=${rest%%:*}; envs=""; [ "$rest" != "$lib" ] && envs=${rest#*:}; }
# variant libraries as absolute paths: tests that start their own processes run them in other directories
setenv() { [ -n "$lib" ] && case "$lib" in /*) export MLG_LIB=$lib ;; *) export MLG_LIB=$GRAFT_REPO_ROOT/$lib ;; esac
           local IFS=,; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; }
for v in ${VARIANTS}; do
  split "$v"
  if [ -n "$TESTS" ]; then
    ( setenv; timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
        $TESTS ) > gpurun_out/ab/tests_$name.log 2>&1 || { echo "tests $name failed"; tail -30 gpurun_out/ab/tests_$name.log; exit 1; }
    echo "tests $name: $(tail -1 gpurun_out/ab/tests_$name.log)"
  fi
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS}; do
    split "$v"
    for m in ${LRN_MODES:-}; do
      out=$( ( setenv; MODE=$m REPS=${REPS:-40} timeout -k 10 300 python scripts/bench_learner.py ) 2> gpurun_out/ab/lrn_${name}_$m.err ) \
          || { echo "learner $name $m failed"; tail -20 gpurun_out/ab/lrn_${name}_$m.err; exit 1; }
      echo "r$r lrn $m $name $out"
    done
    for sc in ${SCRIPTS:-}; do
      out=$( ( setenv; timeout -k 10 300 python $sc ) 2> gpurun_out/ab/script_${name}.err | tail -1 ) \
          || { echo "script $sc $name failed"; tail -20 gpurun_out/ab/script_${name}.err; exit 1; }
      echo "r$r script $(basename $sc) $name $out"
    done
    for m in ${BENCH_MODES:-}; do
      ( setenv; timeout -k 10 300 python bench.py --mode $m --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ) \
          > gpurun_out/ab/bench_${name}_$m.json 2> gpurun_out/ab/bench_${name}_$m.err || { echo "bench $name $m failed"; tail -20 gpurun_out/ab/bench_${name}_$m.err; exit 1; }
      python3 -c "
import json; d=json.load(open('gpurun_out/ab/bench_${name}_$m.json'))
print('r$r bench $m $name', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms', 'kern', round(d['roofline']['avg_kernel_ms'],4), 'len', round(d['mean_episode_len'],2))"
    done
  done
done
