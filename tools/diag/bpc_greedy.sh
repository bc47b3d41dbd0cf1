#!/bin/bash
# Greedy (config 5) bench at rollout blocks per CU, interleaved, twice.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
for b in ${BPC:-2 3 4}; do
  OTH_ROLLOUT_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --workload greedy --no-secondary --steps 30 --warmup 5 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('greedy bpc=$b %.4g env-steps/s  %.4f ms/step' % (d['value'], d['ms_per_step']))" || exit 1
done
done
