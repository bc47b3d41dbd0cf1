#!/bin/bash
# Round-3 session 3: the -m gpu suite on the deferred-terminal rollout loop,
# then A/B/A/B against tools/diag/ab/libhead.so (the fill-order build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
./tools/diag/ab_bench.sh tools/diag/ab/libhead.so --steps 20 --warmup 5 > $O/ab20.log 2>&1 || exit 1
./tools/diag/ab_bench.sh tools/diag/ab/libhead.so --steps 100 --warmup 10 > $O/ab100.log 2>&1 || exit 1
grep -v amdgpu.ids $O/ab20.log $O/ab100.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc -o run -- python3 bench.py --steps 3 --warmup 1 --no-secondary --prewarm-ms 0 > $O/pmc.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O/pmc/run_counter_collection.csv
