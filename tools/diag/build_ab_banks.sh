#!/bin/bash
# Round-3 A/B libraries of the VGPR-bank / batch-tail hand-over experiment
# (DESIGN.md §3), built here on the CPU into tools/diag/ab/:
#   libhead.so       the shipped source, hipcc's allocation
#   libhead_bank.so  the shipped source, tools/vgpr_banks.py on every kernel
#   libho_nobank.so  the hand-over (tools/diag/handoff.patch), hipcc's allocation
#   libnew.so        the hand-over + the bank pass
set -e
cd "$(dirname "$0")/../.."
A=tools/diag/ab
mkdir -p $A
T=$(mktemp -d)
plain() {  # plain hipcc build of $1 -> $2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -I include \
    -Wl,--version-script=subproc_amd/csrc/exports.map -o "$2" "$1" subproc_amd/csrc/td_table.hip
}
plain subproc_amd/csrc/othello.hip $A/libhead.so
python3 tools/vgpr_banks.py --build-lib $A/libhead_bank.so
cp subproc_amd/csrc/othello.hip $T/othello.hip
patch -s $T/othello.hip tools/diag/handoff.patch
cp $T/othello.hip subproc_amd/csrc/_handoff.hip  # (beside bitboard.hpp, for its include)
trap 'rm -f subproc_amd/csrc/_handoff.hip; rm -rf $T' EXIT
plain subproc_amd/csrc/_handoff.hip $A/libho_nobank.so
python3 tools/vgpr_banks.py --build-lib $A/libnew.so subproc_amd/csrc/_handoff.hip
ls -la $A
