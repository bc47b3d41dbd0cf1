#!/bin/bash
# Round profile on the GPU box: rocprofv3 kernel-trace stats of the default bench
# command, then separate PMC passes (FETCH_SIZE, WRITE_SIZE and SQ counters are
# collected in their own runs, as MI355X_MICROARCH.md §rocprofv3 prescribes).
# Usage (via gpurun): ./tools/profile_round.sh r01
set -o pipefail
R=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/prof_$R
mkdir -p $O
# no time-based pre-warm (single-stream launches) in profiled runs: every launch of
# the headline kernel is then a two-stream bench step, as in the bench line
BENCH="bench.py --steps 100 --warmup 100 --prewarm-ms 0 --cpu-games 2000"
# rollout_16M, rollout_1stream and rollout_sharded share the headline kernel and grid: keep them
# out of the per-launch averages
export BENCH_SKIP=rollout_16M,rollout_1stream,rollout_sharded
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $BENCH > $O/kt_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $BENCH > $O/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $BENCH > $O/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $O/sq -o run -- python3 $BENCH > $O/sq.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY --output-format csv -d $O/grbm -o run -- python3 $BENCH > $O/grbm.log 2>&1 || exit 1
python3 tools/profile_summary.py $O > $O/summary.json || exit 1
# hot-loop VALU mix of the same source (the bench's VALU ceiling): copy to profiles/valu_mix.json
python3 tools/valu_mix.py > $O/valu_mix.json || exit 1
cat $O/summary.json
