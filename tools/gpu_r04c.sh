#!/bin/bash
# round-4 iteration: every GPU test, the full bench line, then the step ray-table A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'])
for k,v in d.get('secondary',{}).items(): print(k, v.get('value'), v.get('ms_per_step', v.get('us_per_launch', v.get('ms'))))"
if [ -f build/var/step_rt0.so ]; then
  timeout -k 10 200 python tools/diag/step_ab.py build/var/step_rt0.so build/var/step_rt1.so 5 > $O/step_ab.log 2>&1 || exit 1
  tail -4 $O/step_ab.log
fi
