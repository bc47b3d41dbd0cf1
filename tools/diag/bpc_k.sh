#!/bin/bash
# Headline bench at rollout blocks per CU x streams x timed steps, interleaved, twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
for k in ${KS:-20 100}; do
for cfg in ${CFGS:-3:2 2:2 2:3 3:3 4:2}; do
  b=${cfg%%:*}; s=${cfg##*:}
  OTH_ROLLOUT_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --no-secondary --steps $k --warmup 5 --streams $s 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('k=$k bpc=$b streams=$s %.4g env-steps/s  %.4f ms/step' % (d['value'], d['ms_per_step']))" || exit 1
done
done
done
