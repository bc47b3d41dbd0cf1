#!/bin/bash
# Build the HEAD commit's library into tools/diag/ab/libhead.so (the B side of
# tools/diag/ab_bench.sh), in a temporary worktree.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
W=$(mktemp -d)/wt
git -C "$R" worktree add -q "$W" HEAD
(cd "$W" && python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1)
mkdir -p "$R/tools/diag/ab"
cp "$W/subproc_amd/lib/libsubproc_amd_hip.so" "$R/tools/diag/ab/libhead.so"
git -C "$R" worktree remove --force "$W"
