#!/bin/bash
# Round-3 session 11: ingest tests on the final parse kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s11
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_abi_pair.py -x -q --timeout 120 --timeout-method thread > $O/ingest.log 2>&1 || { tail -40 $O/ingest.log; exit 1; }
tail -2 $O/ingest.log
