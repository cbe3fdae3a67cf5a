#!/bin/bash
# SQ instruction-mix / stall counters of a microbenchmark (BENCH, default scripts/bench_rollout.py), one rocprofv3
# --pmc pass per counter group (<= 8 SQ counters each), counters only. Names not offered by `rocprofv3 -L`
# on this box are dropped before a pass is started.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${OUTNAME:-pmc_sq}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || { echo "rocprofv3 -L failed"; tail -5 $OUT/counters.txt; exit 1; }
run_pass() {
  local name=$1; shift
  local keep=()
  for c in "$@"; do grep -qw "$c" $OUT/counters.txt && keep+=("$c"); done
  echo "pass $name: ${keep[*]}"
  [ ${#keep[@]} -eq 0 ] && return 0
  REPS=3 MLG_BENCH_KERNELS=${KERNELS:-v2} timeout -s KILL 120 rocprofv3 --pmc ${keep[*]} --output-format csv \
      -d "$GRAFT_REPO_ROOT/$OUT/$name" -o run -- python3 ${BENCH:-scripts/bench_rollout.py} > $OUT/$name.json 2> $OUT/$name.err \
      || { echo "pass $name failed"; tail -5 $OUT/$name.err; exit 1; }
}
if [ -n "$PASSES" ]; then
  i=0
  IFS=';' read -ra PS <<< "$PASSES"
  for ps in "${PS[@]}"; do i=$((i+1)); run_pass q$i $ps; done
else
run_pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run_pass p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
run_pass p3 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_FLAT
fi
python3 scripts/parse_pmc.py $OUT ${FILTER:-rollout}
