#!/bin/bash
# A/B/A of the headline bench on one box: the in-tree library (A) against a
# diagnostic build with the same C-ABI (B, $1), swapped in place of A's file.
# Usage (via gpurun): tools/diag/ab_bench.sh tools/diag/ab/libhead.so [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B=$1; shift
L=subproc_amd/lib/libsubproc_amd_hip.so
mkdir -p gpurun_out/ab
cp $L gpurun_out/ab/libA.so || exit 1
run() { timeout -k 10 200 python bench.py --no-secondary "$@" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%s %.4g env-steps/s  %.4f ms/step  launch %.4f ms' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['launch_ms']))" "$TAG"; }
TAG=A run "$@" || exit 1
cp "$B" $L && TAG=B run "$@" || exit 1
cp gpurun_out/ab/libA.so $L && TAG=A run "$@" || exit 1
cp "$B" $L && TAG=B run "$@" || exit 1
cp gpurun_out/ab/libA.so $L
