#!/bin/bash
# TD spec split on the GPU box (diagnostic): its tests, the miss probe under a kernel trace, the TD update rate
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-tdprobe} && mkdir -p $O && timeout -k 10 300 python -u -m pytest tests/test_gpu_td.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/diag/td_spec_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v "^W2026\|^E2026" $O/probe.log | tail -8
timeout -k 10 200 python3 tools/diag/td_trace.py 262144 4 2>&1 | tee $O/td_product.log
