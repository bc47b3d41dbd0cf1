#!/bin/bash
# Round-3 first GPU session: parity of the cut rollout loop, A/B/A/B against the
# round-2 library at the driver's arguments and at 100 steps, VALU PMC of both,
# and the per-launch timeline of a 20-step region.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/s1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
./tools/diag/ab_bench.sh tools/diag/ab/libhead.so --steps 20 --warmup 5 > $O/ab20.log 2>&1 || exit 1
cat $O/ab20.log
./tools/diag/ab_bench.sh tools/diag/ab/libhead.so --steps 100 --warmup 10 > $O/ab100.log 2>&1 || exit 1
cat $O/ab100.log
timeout -k 10 120 python3 tools/diag/timeline.py --steps 20 > $O/timeline20.json 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_new -o run -- python3 bench.py --steps 3 --warmup 1 --no-secondary --prewarm-ms 0 > $O/pmc_new.log 2>&1 || exit 1
python3 tools/pmc_summary.py $O/pmc_new/run_counter_collection.csv > $O/pmc_new.txt 2>&1
cp subproc_amd/lib/libsubproc_amd_hip.so $O/libnew.so && cp tools/diag/ab/libhead.so subproc_amd/lib/libsubproc_amd_hip.so || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_old -o run -- python3 bench.py --steps 3 --warmup 1 --no-secondary --prewarm-ms 0 > $O/pmc_old.log 2>&1
rc=$?
cp $O/libnew.so subproc_amd/lib/libsubproc_amd_hip.so && rm $O/libnew.so
[ $rc -eq 0 ] || exit 1
python3 tools/pmc_summary.py $O/pmc_old/run_counter_collection.csv > $O/pmc_old.txt 2>&1
cat $O/pmc_new.txt $O/pmc_old.txt | cut -c1-300
