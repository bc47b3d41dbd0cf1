#!/bin/bash
# Round-3 session: the eval policy's child fill order 7-9-8 (9 same-bank
# v_bitop3_b32 in its child loop, in-mix mean 3.568) against the shipped 8-7-9
# (13, 3.589).  Eval parity tests on it, then the bench's eval line, three passes.
#   (tools/diag/ab/libev798.so: build_variant.py + asm_ident.py with moves<798> in child_key)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/evalorder
mkdir -p $O
L=subproc_amd/lib/libsubproc_amd_hip.so
cp $L $O/libshipped.so || exit 1
cp tools/diag/ab/libev798.so $L || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py tests/test_gpu_td.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { cp $O/libshipped.so $L; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cat > $O/ev.py <<'PY'
import sys, time, torch
sys.path.insert(0, ".")
from subproc_amd import ops
dev = torch.device("cuda:0")
for _ in range(3): ops.rollout(1 << 20, seed=1, policy="eval", device=dev)
torch.cuda.synchronize()
t = time.perf_counter(); steps = 0
for i in range(10):
    r = ops.rollout(1 << 20, seed=100 + i, policy="eval", device=dev)
    steps += int(r.hist[132])
torch.cuda.synchronize()
dt = time.perf_counter() - t
print("%s eval %.4g env-steps/s (%.3f ms per launch, one stream)" % (sys.argv[1], steps / dt, dt / 10 * 1e3))
PY
for pass in 1 2 3; do
  for v in shipped ev798; do
    case $v in shipped) cp $O/libshipped.so $L;; *) cp tools/diag/ab/lib$v.so $L;; esac || exit 1
    timeout -k 10 120 python $O/ev.py $v >> $O/ab.log 2>&1 || { cp $O/libshipped.so $L; cat $O/ab.log; exit 1; }
  done
done
cp $O/libshipped.so $L
grep -v amdgpu.ids $O/ab.log
