#!/bin/bash
# Round-3 session 9: book ingest (oth_book_parse, oth_td_updates_records) --
# the GPU suite with the new tests, then the bench line's book_emitter section.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s9
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_ingest.py -x -v --timeout 120 --timeout-method thread > $O/ingest.log 2>&1 || { tail -40 $O/ingest.log; exit 1; }
tail -3 $O/ingest.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); print(d['value']); print(json.dumps(d['secondary']['book_emitter'], indent=0))"
