#!/bin/bash
# Headline occupancy sweep on one box (round 6): bench.py's config-3 line at the
# driver's --steps 20 --warmup 5 for random-policy blocks per CU x streams x the
# hand-over K, alternating, REPS passes.
# Usage (GPU box): [CFGS="b,s,k b,s,k ..."] tools/gpu_occ_sweep.sh OUT [REPS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; REPS=${2:-2}
mkdir -p $O
line() { python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print('%-16s %.4e  %.4f ms/step  launch %.4f ms' % (sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['launch_ms']))" "$@"; }
for rep in $(seq $REPS); do
  for cfg in ${CFGS:-3,2,16 4,2,16 3,3,16 4,3,16 2,3,16 3,2,8}; do
    set -- ${cfg//,/ }
    tag=b$1s$2k$3
    OTH_ROLLOUT_BLOCKS_PER_CU=$1 OTH_HANDOFF_K=$3 timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-secondary --streams $2 > $O/${tag}_$rep.log 2>&1 || { tail -5 $O/${tag}_$rep.log; exit 1; }
    line $O/${tag}_$rep.log $tag | tee -a $O/sweep.txt
  done
done
