#!/bin/bash
# round-4 iteration: the kernels touched (1-ply choice, TD map) -> their GPU tests, then the full bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r04c}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runner.py tests/test_gpu_td.py tests/test_gpu_ingest.py tests/test_gpu_facade.py tests/test_gpu_engine.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'])
for k,v in d.get('secondary',{}).items(): print(k, v.get('value'), v.get('ms_per_step', v.get('us_per_launch', v.get('ms'))))"
