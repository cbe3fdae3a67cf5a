#!/bin/bash
# Counter evidence for the rollout kernels at the current commit: per mode (ai = v7, league = sp7,
# refil = refil_rollout), separate rocprofv3 --pmc passes, counters only (no trace domains):
#   FETCH_SIZE | WRITE_SIZE (HBM bytes; they cannot share a pass) | 3 SQ passes (<= 8 SQ + 1 GRBM counters each)
# then scripts/parse_counters.py -> gpurun_out/counters/counters.json (copied to profiles/counters.json).
# COMMIT names the profiled commit (the box has no .git); HBM_ONLY=1 runs the two HBM passes only.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/counters
mkdir -p $OUT
pass() {  # mode name counters...
  local mode=$1 name=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/$mode/$name" -o run \
      -- python3 bench.py --mode $mode --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline \
      > $OUT/$mode/$name.json 2> $OUT/$mode/$name.err || { echo "pass $mode/$name failed"; tail -5 $OUT/$mode/$name.err; exit 1; }
  echo "pass $mode/$name ok"
}
for m in ${MODES:-ai league refil}; do
  mkdir -p $OUT/$m
  pass $m fetch FETCH_SIZE
  pass $m write WRITE_SIZE
  [ -n "$HBM_ONLY" ] && continue
  pass $m sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
  pass $m sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
  pass $m sq3 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE
done
python3 scripts/parse_counters.py $OUT "${COMMIT:-unknown}" ${MERGE:-} > $OUT/counters.json || exit 1
cat $OUT/counters.json
