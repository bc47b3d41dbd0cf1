#!/bin/bash
# 1-ply policies: forced moves (one legal move) played unscored (OTH_COOP_FORCED=1)
# against scoring their one child (=0), one box (diagnostic, round 5):
# policy_ab.py times (histograms compared), the children counts, then one PMC
# pass per library and policy (3 launches of 1M games each).
# Usage (GPU box): tools/diag/forced_ab.sh OUT OFF.so ON.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python3 tools/diag/policy_ab.py "$@" --policies greedy,eval --reps 7 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 200 python3 tools/diag/eval_pmc.py $1 --greedy --children > $O/children_greedy.log 2>&1 || { tail -5 $O/children_greedy.log; exit 1; }
timeout -k 10 200 python3 tools/diag/eval_pmc.py $1 --children > $O/children_eval.log 2>&1 || { tail -5 $O/children_eval.log; exit 1; }
cat $O/children_greedy.log $O/children_eval.log
for L in "$@"; do
  b=$(basename $L .so)
  for pol in greedy eval; do
    flag=""; [ $pol = greedy ] && flag=--greedy
    timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/$b.$pol -o run -- python3 tools/diag/eval_pmc.py $L $flag > $O/$b.$pol.log 2>&1 || { echo "pmc $b $pol failed"; tail -3 $O/$b.$pol.log; exit 1; }
  done
done
python3 - $O "$@" <<'PY'
import csv, glob, os, sys, collections
O = sys.argv[1]
for L in sys.argv[2:]:
    b = os.path.basename(L)[:-3]
    for pol, kern in (("greedy", "rollout_kernel<1"), ("eval", "rollout_kernel<2")):
        tot = collections.defaultdict(list)
        for f in glob.glob("%s/%s.%s/**/*counter_collection.csv" % (O, b, pol), recursive=True):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    tot[r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(b, pol, {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(tot.items())})
PY
