#!/bin/bash
# Round-3 session 10: the LDS-staged parse path -- ingest tests, then the
# bench's book_emitter section.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s10
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_books.py tests/test_gpu_td.py -x -q --timeout 120 --timeout-method thread > $O/ingest.log 2>&1 || { tail -40 $O/ingest.log; exit 1; }
tail -2 $O/ingest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); b=d['secondary']['book_emitter']; print({k:(round(v['us'],1), round(v['achieved_gbs'])) for k,v in b.items() if isinstance(v,dict)})"
