#!/bin/bash
# (libraries: tools/diag/build_ab_banks.sh, run here first)
# Round-3 session: the batch-tail hand-over on the VGPR-bank pass
# (subproc_amd/csrc/vgpr_banks.py).  GPU suite on the in-tree library, then the
# headline at the driver's arguments, two passes over four builds:
#   new       in-tree: hand-over + bank pass
#   head      HEAD (no hand-over, hipcc's allocation)
#   head_bank HEAD + bank pass
#   ho_nobank hand-over, hipcc's allocation
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/banks
mkdir -p $O
L=subproc_amd/lib/libsubproc_amd_hip.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cp $L $O/libshipped.so || exit 1
run() { timeout -k 10 200 env $KENV python bench.py --no-secondary --steps 20 --warmup 5 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-9s %.4g env-steps/s  %.4f ms/step  launch %.4f ms' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['launch_ms']))" "$1"; }
for pass in 1 2; do
  for v in new head head_bank ho_nobank new_k4 new_k12 new_k16; do
    KENV=OTH_HANDOFF_K=${v#new_k}; [ "${v#new_k}" = "$v" ] && KENV=
    case $v in new*) cp tools/diag/ab/libnew.so $L;; *) cp tools/diag/ab/lib$v.so $L;; esac || exit 1
    run $v >> $O/ab.log 2>&1 || { cp $O/libshipped.so $L; cat $O/ab.log; exit 1; }
  done
done
cp $O/libshipped.so $L
grep -v amdgpu.ids $O/ab.log
