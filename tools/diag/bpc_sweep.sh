#!/bin/bash
# Headline bench at several rollout blocks per CU (OTH_ROLLOUT_BLOCKS_PER_CU), twice each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
for b in ${BPC:-4 5 6 7}; do
  OTH_ROLLOUT_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --no-secondary --steps 50 --warmup 5 ${BENCH_ARGS} 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bpc=$b %.4g env-steps/s  %.4f ms/step' % (d['value'], d['ms_per_step']))" || exit 1
done
done
