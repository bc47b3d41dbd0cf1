#!/bin/bash
# TD pipeline on the GPU box (diagnostic): its tests, then a kernel trace of
# three 262,144-game updates (tools/diag/td_trace.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-tdcheck} && mkdir -p $O || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_td.py tests/test_gpu_ingest.py tests/test_gpu_abi_pair.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { grep -B5 -A30 "Error\|FAIL" $O/pytest.log | head -60; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/diag/td_trace.py 262144 3 > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
grep batch $O/log
