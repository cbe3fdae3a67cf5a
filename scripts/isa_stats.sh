#!/bin/bash
# isa_stats.sh [extra hipcc flags]: device asm of rollout.hip; register use and step-loop instruction mix of the
# static 5v5 v7 kernel (rollout_v2_kernel<64, true, 5, 10>). Analysis aid only.
cd "$(dirname "$0")/../ma-league_amd" || exit 1
out=${OUT:-/tmp/rollout_isa.s}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Wno-unused-function --cuda-device-only -S \
    "$@" csrc/rollout.hip -o $out 2>/dev/null || exit 1
python3 ../scripts/isa_stats.py "$out"
