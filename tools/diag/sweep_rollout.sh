#!/bin/bash
# Launch-geometry sweep of the rollout kernel (diagnostic build) — run on the GPU box.
set -o pipefail
for bpc in ${BPC:-1 2 3 4}; do
  echo "== blocks_per_cu=$bpc"
  OTH_ROLLOUT_BLOCKS_PER_CU=$bpc timeout -k 10 60 ./tools/diag/rollout_diag ${N:-1048576} 3 | tail -1 || exit 1
done
