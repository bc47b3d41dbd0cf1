#!/bin/bash
# Round-3 session 4: VALU issue costs of further instruction classes
# (valu_rate5), and the single-stream rollout at 3 vs 5 blocks per CU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 120 ./tools/diag/valu_rate5 > $O/valu_rate5.txt 2>&1 || exit 1
cat $O/valu_rate5.txt
run() { timeout -k 10 200 python bench.py --no-secondary --streams 1 --steps 20 --warmup 5 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%s %.4g env-steps/s  %.4f ms/step' % (sys.argv[1], d['value'], d['ms_per_step']))" "$1"; }
for k in 1 2; do
  OTH_ROLLOUT_BLOCKS_PER_CU=3 run "1stream bpc3" >> $O/bpc.log 2>&1 || exit 1
  OTH_ROLLOUT_BLOCKS_PER_CU=5 run "1stream bpc5" >> $O/bpc.log 2>&1 || exit 1
  OTH_ROLLOUT_BLOCKS_PER_CU=7 run "1stream bpc7" >> $O/bpc.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/bpc.log
