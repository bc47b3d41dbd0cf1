#!/bin/bash
# eval-policy A/B on one box (diagnostic): the 24-bit-multiply eval build
# against the plain-multiply one and round 3's choice, the TD and eval tests,
# and the TD update rate
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-evalab} && mkdir -p $O || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_td.py tests/test_gpu_ingest.py tests/test_gpu_abi_pair.py tests/test_gpu_parity.py tests/test_gpu_runner.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { grep -B5 -A30 "Error\|FAIL" $O/pytest.log | head -60; exit 1; }
timeout -k 10 200 python3 tools/diag/td_trace.py 262144 4 2>&1 | tee $O/td_product.log
timeout -k 10 400 python tools/diag/policy_ab.py build/var/mul24.so build/var/mul32.so build/var/r03coop.so --policies eval,greedy --reps 7 > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
cat $O/ab.log
