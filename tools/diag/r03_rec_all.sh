#!/bin/bash
# Round 3: record staging for the 1-ply policies too (OTH_REC_ALL build in
# tools/diag/ab/librecall.so) against the in-tree library (random only):
# the tests that record moves on the candidate, then record rollouts timed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/recall
mkdir -p $O
L=subproc_amd/lib/libsubproc_amd_hip.so
cp $L $O/libA.so || exit 1
timeout -k 10 200 python tools/diag/record_policies.py A > $O/a1.log 2>&1 || exit 1
cp tools/diag/ab/librecall.so $L || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_runner.py tests/test_gpu_books.py tests/test_gpu_parity.py tests/test_gpu_abi_pair.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; cp $O/libA.so $L; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/diag/record_policies.py B > $O/b1.log 2>&1 || { cp $O/libA.so $L; exit 1; }
cp $O/libA.so $L
timeout -k 10 200 python tools/diag/record_policies.py A > $O/a2.log 2>&1 || exit 1
grep -h "per launch" $O/a1.log $O/b1.log $O/a2.log
