#!/bin/bash
# Round 3: the TD pair sort at 9-bit digits -- TD / ABI-pair / ingest tests and
# the bench's TD line (twice).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/tdsort
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_td.py tests/test_gpu_ingest.py tests/test_gpu_abi_pair.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench$k.json 2> $O/bench$k.err || { tail -20 $O/bench$k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench$k.json').read().splitlines()[-1]); print(d['value'], d['secondary']['td_state_map']['value'], d['secondary']['td_state_map']['ms'])"
done
