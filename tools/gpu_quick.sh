#!/bin/bash
# Quick GPU iteration loop: parity tests, launch-geometry sweep, bench, VALU PMC.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/q
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/q/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/q/pytest.log
tail -2 gpurun_out/q/pytest.log
grep -q "pytest rc=0" gpurun_out/q/pytest.log || exit 1
BPC="${BPC:-2 3 4 5}" ./tools/diag/sweep_rollout.sh > gpurun_out/q/sweep.log 2>&1 || exit 1
cut -c1-200 gpurun_out/q/sweep.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/q/bench.log 2>&1 || exit 1
tail -1 gpurun_out/q/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'], d['ms_per_step']); print({k: (v['value'], v.get('roofline',{}).get('frac')) for k,v in d.get('secondary',{}).items()})"
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/q/pmc -o run -- python3 bench.py --steps 3 --warmup 1 --no-secondary > gpurun_out/q/pmc.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/q/pmc/run_counter_collection.csv
