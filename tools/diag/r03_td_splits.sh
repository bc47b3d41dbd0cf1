#!/bin/bash
# Round 3: merge-path splits from a partition kernel and staged lookup outputs
# (td_table.hip) -- TD and ABI-pair tests, the bench's td_state_map line, then
# the round profile for the lookup / merge HBM traffic.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/tds
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_td.py tests/test_gpu_abi_pair.py tests/test_gpu_ingest.py tests/test_gpu_books.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print(d['value'], json.dumps(d['secondary']['td_state_map']))"
./tools/profile_round.sh r03 > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo profiled
