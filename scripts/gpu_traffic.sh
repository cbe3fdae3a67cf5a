#!/bin/bash
# HBM traffic of the dominant kernel from PMC counters: two separate rocprofv3 --pmc passes (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950), counters only -- no trace domains. Then the bench with the result.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
MODE=${MODE:-ai}
OUT=gpurun_out/pmc_$MODE
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/$c" -o run -- python3 bench.py --mode $MODE --steps 4 --warmup 2 --no-cpu-baseline > $OUT/$c.json 2> $OUT/$c.err || { echo "pmc $c failed"; tail -5 $OUT/$c.err; exit 1; }
done
python3 scripts/parse_traffic.py $OUT > $OUT/traffic.json || exit 1
cat $OUT/traffic.json
