#!/bin/bash
# Round-3 session: the random loop's flips by one joint reversal
# (bitboard.hpp flips_col_joint, OTH_JOINT_FLIPS; fill order 8-9-7) against
# the shipped library (four run sets reversed whole).  Rollout parity tests on
# it, then the headline at the driver's arguments, three passes.
#   (tools/diag/ab/libjoint.so: build_variant.py + asm_ident.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/joint
mkdir -p $O
L=subproc_amd/lib/libsubproc_amd_hip.so
cp $L $O/libshipped.so || exit 1
cp tools/diag/ab/libjoint.so $L || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py tests/test_gpu_abi_pair.py tests/test_gpu_books.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { cp $O/libshipped.so $L; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { timeout -k 10 200 python bench.py --no-secondary --steps 20 --warmup 5 ${EXTRA} | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-16s %.4g env-steps/s  %.4f ms/step  launch %.4f ms' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['launch_ms']))" "$1"; }
for pass in 1 2 3; do
  for v in shipped joint; do
    case $v in shipped) cp $O/libshipped.so $L;; *) cp tools/diag/ab/lib$v.so $L;; esac || exit 1
    run $v >> $O/ab.log 2>&1 || { cp $O/libshipped.so $L; cat $O/ab.log; exit 1; }
  done
done
cp $O/libshipped.so $L
grep -v amdgpu.ids $O/ab.log
