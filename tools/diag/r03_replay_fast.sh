#!/bin/bash
# Round 3: the replay's fast path (flips_carry for a recorded move that flips,
# the analysis only for passes, illegal codes and last positions) -- the
# replay / books / TD / ABI-pair tests, then the bench's book_emitter line
# (twice).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/replay
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_books.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench$k.json 2> $O/bench$k.err || { tail -20 $O/bench$k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench$k.json').read().splitlines()[-1]); b=d['secondary']['book_emitter']; print(d['value'], {k:(round(v['us'],1), round(v['achieved_gbs'])) for k,v in b.items() if isinstance(v,dict)})"
done
