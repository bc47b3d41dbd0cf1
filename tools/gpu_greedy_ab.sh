#!/bin/bash
# Greedy / eval A/B on one box (round 6): tools/diag/policy_ab.py one-stream
# launches alternating over the libraries, then bench.py's greedy line (two
# streams, config 5) per library, alternating, two passes.
# Usage (GPU box): tools/gpu_greedy_ab.sh OUT LIB...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python3 tools/diag/policy_ab.py "$@" --policies greedy,eval --reps 5 > $O/policy_ab.log 2>&1 || { tail -5 $O/policy_ab.log; exit 1; }
tail -8 $O/policy_ab.log
for rep in 1 2; do
  for L in "$@"; do
    timeout -k 10 200 python3 bench.py --workload greedy --steps 20 --warmup 5 --no-secondary --lib $L > $O/g_$(basename $L)_$rep.log 2>&1 || { tail -5 $O/g_$(basename $L)_$rep.log; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print('%-10s greedy 2-stream %.4e  %.4f ms/step' % (sys.argv[2], d['value'], d['ms_per_step']))" $O/g_$(basename $L)_$rep.log $(basename $L) | tee -a $O/greedy.txt
  done
done
# per library: the greedy kernel's HBM write bytes (one WRITE_SIZE pass)
for L in "$@"; do
  PROBE_LIB=$L timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$(basename $L) -o run -- python3 tools/diag/lds_probe.py greedy > $O/w_$(basename $L).log 2>&1 || { tail -5 $O/w_$(basename $L).log; exit 1; }
  python3 - $O/w_$(basename $L) $(basename $L) <<'PY'
import csv, glob, sys, re
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if re.search(r"rollout_kernel<1, false, false>", r["Kernel_Name"])]
print("%-10s greedy WRITE_SIZE %.2f MB per launch" % (sys.argv[2], sum(v) / len(v) * 1024 / 1e6))
PY
done
