#!/bin/bash
# GPU tests (all, or the files given in $TESTS), then the A/B/A/B headline
# bench of the in-tree library against tools/diag/ab/libhead.so.
# Usage (via gpurun): TESTS="tests/test_gpu_parity.py" tools/diag/ab_check.sh tag [bench args]
T=${1:-ab}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 bash tools/diag/ab_bench.sh tools/diag/ab/libhead.so "$@" 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
