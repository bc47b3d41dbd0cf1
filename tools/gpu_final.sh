#!/bin/bash
# Round close on one GPU box: the TD check and trace, every -m gpu test, smoke,
# the bench at the driver's arguments, the round profile of the same build,
# and the bench again with that profile in place (its PMC figures current).
# Usage (via gpurun): ./tools/gpu_final.sh r04
R=${1:-r04}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
./tools/gpu_td_check.sh ${R}_td || exit 1
BENCH_ARGS="--steps 20 --warmup 5" ./tools/gpu_check.sh ${R}_check || exit 1
./tools/profile_round.sh $R > /dev/null || exit 1
cp gpurun_out/prof_$R/summary.json profiles/${R}_profile_summary.json || exit 1
mkdir -p gpurun_out/${R}_bench2
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${R}_bench2/bench.log 2>&1 || { tail -5 gpurun_out/${R}_bench2/bench.log; exit 1; }
tail -1 gpurun_out/${R}_bench2/bench.log | cut -c1-400
