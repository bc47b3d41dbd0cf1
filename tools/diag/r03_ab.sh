#!/bin/bash
# A/B/A/B of the in-tree library against tools/diag/ab/libhead.so: the headline
# at the driver's arguments and at 100 steps, and the greedy workload.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab3
mkdir -p $O
./tools/diag/ab_bench.sh tools/diag/ab/libhead.so --steps 20 --warmup 5 > $O/ab20.log 2>&1 || exit 1
./tools/diag/ab_bench.sh tools/diag/ab/libhead.so --steps 100 --warmup 10 > $O/ab100.log 2>&1 || exit 1
./tools/diag/ab_bench.sh tools/diag/ab/libhead.so --workload greedy --steps 10 --warmup 2 > $O/abgreedy.log 2>&1 || exit 1
grep -v amdgpu.ids $O/ab20.log $O/ab100.log $O/abgreedy.log
