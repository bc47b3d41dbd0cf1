#!/bin/bash
# TD kernels' HBM traffic (diagnostic, round 5): FETCH_SIZE and WRITE_SIZE
# passes (separate runs) over tools/diag/td_trace.py; per-kernel averages by
# tools/pmc_summary.py's rules are left to the reader (td_pmc_digest.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-tdpmc} && mkdir -p $O || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/diag/td_trace.py 262144 3 > $O/kt.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/diag/td_trace.py 262144 3 > $O/fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/diag/td_trace.py 262144 3 > $O/write.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq -o run -- python3 tools/diag/td_trace.py 262144 3 > $O/sq.log 2>&1 || exit 1
