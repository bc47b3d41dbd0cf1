#!/bin/bash
# Round-3 session 6: the two-stream headline at 2/3/4 blocks per CU and 2/3
# streams with the round-3 kernel (20 timed steps, two passes each).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s6
mkdir -p $O
run() { timeout -k 10 200 python bench.py --no-secondary --steps 20 --warmup 5 "${@:2}" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%s %.4g env-steps/s  %.4f ms/step' % (sys.argv[1], d['value'], d['ms_per_step']))" "$1"; }
for k in 1 2; do
  for b in 2 3 4; do
    OTH_ROLLOUT_BLOCKS_PER_CU=$b run "bpc$b s2" --streams 2 >> $O/sweep.log 2>&1 || exit 1
  done
  OTH_ROLLOUT_BLOCKS_PER_CU=2 run "bpc2 s3" --streams 3 >> $O/sweep.log 2>&1 || exit 1
  OTH_ROLLOUT_BLOCKS_PER_CU=3 run "bpc3 s3" --streams 3 >> $O/sweep.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/sweep.log
