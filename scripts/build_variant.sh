#!/bin/bash
# build_variant.sh NAME "-DFLAG=..." : libmaleague variant into ma-league_amd/maleague/_lib/variants/NAME.so
set -e
cd "$(dirname "$0")/../ma-league_amd"
mkdir -p maleague/_lib/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-function $2 csrc/*.hip -o maleague/_lib/variants/$1.so
