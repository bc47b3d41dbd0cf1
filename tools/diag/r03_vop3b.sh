#!/bin/bash
# Round-3 session: VOP3 encodings at source level (bitboard.hpp and2/or2/sh32/
# bfrev32) against the assembly pass (tools/diag/vop3_promote.py).  Rollout
# parity tests on the source build, then the headline at the driver's
# arguments and greedy, two passes:
#   shipped   in-tree library (HEAD: VOP2 and/or, VOP1 bfrev)
#   vop3      HEAD + the assembly pass over the rollout kernels
#   src       the source-level VOP3 build (random loop fill order 7-8-9)
#   srcvop3   the source-level build + the assembly pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/vop3b
mkdir -p $O
L=subproc_amd/lib/libsubproc_amd_hip.so
cp $L $O/libshipped.so || exit 1
cp tools/diag/ab/libsrc.so $L || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py tests/test_gpu_board_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { cp $O/libshipped.so $L; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp $O/libshipped.so $L
run() { timeout -k 10 200 python bench.py --no-secondary --steps 20 --warmup 5 ${EXTRA} | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-16s %.4g env-steps/s  %.4f ms/step  launch %.4f ms' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['launch_ms']))" "$1"; }
put() { case $1 in shipped) cp $O/libshipped.so $L;; *) cp tools/diag/ab/lib$1.so $L;; esac; }
for pass in 1 2; do
  for v in shipped vop3 src srcvop3; do
    put $v || exit 1
    run $v >> $O/ab.log 2>&1 || { cp $O/libshipped.so $L; cat $O/ab.log; exit 1; }
  done
done
for v in shipped src srcvop3; do
  put $v || exit 1
  EXTRA="--workload greedy" run greedy_$v >> $O/ab.log 2>&1 || { cp $O/libshipped.so $L; cat $O/ab.log; exit 1; }
done
cp $O/libshipped.so $L
grep -v amdgpu.ids $O/ab.log
