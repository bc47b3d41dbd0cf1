#!/bin/bash
# Round-3 session 7: the batch-tail hand-over.  GPU suite on the new library,
# then A/B/A/B against HEAD's build (tools/diag/ab/libhead.so) at the driver's
# arguments, and the new library with the hand-over disabled (OTH_HANDOFF_K=0).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s7
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
./tools/diag/ab_bench.sh tools/diag/ab/libhead.so --steps 20 --warmup 5 > $O/ab20.log 2>&1 || exit 1
run() { timeout -k 10 200 python bench.py --no-secondary --steps 20 --warmup 5 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%s %.4g env-steps/s  %.4f ms/step  launch %.4f ms' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['launch_ms']))" "$1"; }
OTH_HANDOFF_K=0 run K0 >> $O/k.log 2>&1 || exit 1
OTH_HANDOFF_K=4 run K4 >> $O/k.log 2>&1 || exit 1
run K8 >> $O/k.log 2>&1 || exit 1
OTH_HANDOFF_K=0 run K0 >> $O/k.log 2>&1 || exit 1
OTH_HANDOFF_K=4 run K4 >> $O/k.log 2>&1 || exit 1
run K8 >> $O/k.log 2>&1 || exit 1
grep -v amdgpu.ids $O/ab20.log $O/k.log
