#!/bin/bash
# Replay kernel: parity tests touching it, timing, and FETCH/WRITE PMC passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/replay
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_board_api.py tests/test_gpu_books.py tests/test_gpu_abi_pair.py tests/test_gpu_td.py tests/test_gpu_engine.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/diag/replay_bw.py > $O/time.log 2>&1 || exit 1
cat $O/time.log
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/diag/replay_bw.py > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/diag/replay_bw.py > $O/write.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/diag/replay_bw.py > $O/kt.log 2>&1 || exit 1
python3 tools/pmc_summary.py --match=replay $O/fetch/run_counter_collection.csv $O/write/run_counter_collection.csv
grep -i replay $O/kt/run_kernel_stats.csv | cut -c1-300
