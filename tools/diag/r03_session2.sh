#!/bin/bash
# Round-3 GPU session 2: the -m gpu suite (packed replay rows, graph words, the
# two-rank bench line), the pre-warm A/B at the driver's arguments, and one
# full bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
run() { timeout -k 10 200 python bench.py --no-secondary --steps 20 --warmup 5 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%s %.4g env-steps/s  %.4f ms/step  step %.4f launch %.4f ms' % (sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['step_ms'], d['roofline']['launch_ms']))" "$1"; }
for k in 1 2 3; do
  BENCH_PREWARM_SYNC=1 run sync >> $O/prewarm.log 2>&1 || exit 1
  run continuous >> $O/prewarm.log 2>&1 || exit 1
done
cat $O/prewarm.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
tail -c 3000 $O/bench_driver.json
