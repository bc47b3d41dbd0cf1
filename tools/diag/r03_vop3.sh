#!/bin/bash
# Round-3 session: VOP3 encodings of the rollout kernels' VOP1/VOP2 VALU
# (tools/diag/vop3_promote.py, valu_rate7.cpp).  The rollout parity tests on
# the promoted library, then the headline at the driver's arguments, two passes:
#   shipped  in-tree library
#   asm      hipcc's assembly re-assembled unchanged (the route's control)
#   vop3     promoted
# (libraries, built here first: python tools/diag/build_variant.py tools/diag/ab/libasm.so
#  tools/diag/asm_ident.py; ... libvop3.so tools/diag/vop3_promote.py rollout_kernel)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/vop3
mkdir -p $O
L=subproc_amd/lib/libsubproc_amd_hip.so
cp $L $O/libshipped.so || exit 1
cp tools/diag/ab/libvop3.so $L || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { cp $O/libshipped.so $L; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cp $O/libshipped.so $L
run() { timeout -k 10 200 python bench.py --no-secondary --steps 20 --warmup 5 ${EXTRA} | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-9s %.4g env-steps/s  %.4f ms/step  launch %.4f ms' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['launch_ms']))" "$1"; }
for pass in 1 2; do
  for v in shipped asm vop3; do
    case $v in shipped) cp $O/libshipped.so $L;; *) cp tools/diag/ab/lib$v.so $L;; esac || exit 1
    run $v >> $O/ab.log 2>&1 || { cp $O/libshipped.so $L; cat $O/ab.log; exit 1; }
  done
done
for v in shipped vop3; do
  case $v in shipped) cp $O/libshipped.so $L;; *) cp tools/diag/ab/lib$v.so $L;; esac || exit 1
  EXTRA="--workload greedy" run greedy_$v >> $O/ab.log 2>&1 || { cp $O/libshipped.so $L; cat $O/ab.log; exit 1; }
done
cp $O/libshipped.so $L
grep -v amdgpu.ids $O/ab.log
