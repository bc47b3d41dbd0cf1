#!/bin/bash
# batch-tail hand-over A/B on one box (diagnostic, round 5): bench.py's headline
# line at the driver's --steps 20 --warmup 5 with the OTH_HANDOFF=0 build and
# the shipped (hand-over) build at several K, three passes; then policy_ab.py's
# one-stream launches (random) for the same two builds.
# Usage (GPU box): tools/gpu_handoff_ab.sh OUT OFF.so ON.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; OFF=$2; ON=$3
mkdir -p $O
line() { python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print('%-12s %.4e  %.4f ms' % (sys.argv[2], d['value'], d['ms_per_step']))" "$@"; }
for rep in 1 2 3; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-secondary --lib $OFF > $O/off_$rep.log 2>&1 || exit 1
  line $O/off_$rep.log off
  for k in 8 12 16; do
    OTH_HANDOFF_K=$k timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-secondary --lib $ON > $O/on${k}_$rep.log 2>&1 || exit 1
    line $O/on${k}_$rep.log on_k$k
  done
done
timeout -k 10 240 python3 tools/diag/policy_ab.py $OFF $ON --policies random --reps 7 > $O/policy_ab.log 2>&1 || exit 1
tail -3 $O/policy_ab.log
