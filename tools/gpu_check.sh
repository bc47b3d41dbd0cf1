#!/bin/bash
# Round check on the GPU box: every -m gpu test, smoke(), and the default bench line.
# Usage (via gpurun): ./tools/gpu_check.sh [tag]
T=${1:-check}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS} > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-600
