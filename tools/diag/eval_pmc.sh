#!/bin/bash
# eval policy: chunked choice (round 4/5) against round 3's surplus list, one
# box (diagnostic): policy_ab.py times, then per library two PMC passes of
# eval_pmc.py (3 launches of 1M games each).  Usage: tools/diag/eval_pmc.sh OUT LIB.so ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python3 tools/diag/policy_ab.py "$@" --policies eval --reps 7 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
tail -$(( $# + 1 )) $O/ab.log
timeout -k 10 200 python3 tools/diag/eval_pmc.py $1 --children > $O/children.log 2>&1 || { tail -5 $O/children.log; exit 1; }
cat $O/children.log
for L in "$@"; do
  b=$(basename $L .so)
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/$b.p1 -o run -- python3 tools/diag/eval_pmc.py $L > $O/$b.p1.log 2>&1 || { echo "pmc1 $b failed"; tail -3 $O/$b.p1.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU --output-format csv -d $O/$b.p2 -o run -- python3 tools/diag/eval_pmc.py $L > $O/$b.p2.log 2>&1 || { echo "pmc2 $b failed"; tail -3 $O/$b.p2.log; exit 1; }
done
python3 - $O "$@" <<'PY'
import csv, glob, os, sys, collections
O = sys.argv[1]
for L in sys.argv[2:]:
    b = os.path.basename(L)[:-3]
    tot = collections.defaultdict(list)
    for p in ("p1", "p2"):
        for f in glob.glob("%s/%s.%s/**/*counter_collection.csv" % (O, b, p), recursive=True):
            for r in csv.DictReader(open(f)):
                if "rollout_kernel<2" in r["Kernel_Name"]:
                    tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(b, {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(tot.items())})
PY
