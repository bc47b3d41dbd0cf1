#!/bin/bash
# Replay kernel: SQ instruction / wait counters (two --pmc passes, each its own run).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/replay_sq
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $O/sq -o run -- python3 tools/diag/replay_bw.py > $O/sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU --output-format csv -d $O/grbm -o run -- python3 tools/diag/replay_bw.py > $O/grbm.log 2>&1 || exit 1
python3 tools/pmc_summary.py --match=replay $O/sq/run_counter_collection.csv $O/grbm/run_counter_collection.csv
