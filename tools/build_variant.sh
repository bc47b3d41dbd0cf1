#!/bin/bash
# Build the HIP library from a copy of the sources with extra flags (A/B builds
# for tools/diag/policy_ab.py and bench.py --lib; never the shipped library).
# Usage: tools/build_variant.sh OUT.so SRC_DIR [hipcc flags...]
#   SRC_DIR holds othello.hip, td_table.hip, bitboard.hpp, td_skey.hpp
OUT=$1; SRC=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
exec /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -pragma-unroll-threshold=200000 \
  -I "$R/include" -Wl,--version-script="$R/subproc_amd/csrc/exports.map" "$@" -o "$OUT" "$SRC/othello.hip" "$SRC/td_table.hip"
