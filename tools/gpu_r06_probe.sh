#!/bin/bash
# Round 6 probes on one box: (1) the TD EMA fork A/B inside the full bench (one
# stream pool shared by every bench line), alternating, two passes; (2) one
# LDS PMC pass over the three rollout policies (SQ_LDS_BANK_CONFLICT etc.).
# Usage (GPU box): tools/gpu_r06_probe.sh OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
mkdir -p $O
td() { python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; t=d['secondary']['td_state_map']; print('%-8s headline %.4e  td %.3f ms (%.3f-%.3f)' % (sys.argv[2], d['value'], t['ms'], t['ms_min'], t['ms_max']))" "$@"; }
for rep in 1 2; do
  for f in 0 1; do
    OTH_TD_EMA_FORK=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/fork${f}_$rep.log 2>&1 || { tail -5 $O/fork${f}_$rep.log; exit 1; }
    td $O/fork${f}_$rep.log fork$f | tee -a $O/fork.txt
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d $O/lds -o run -- python3 tools/diag/lds_probe.py > $O/lds.log 2>&1 || { tail -5 $O/lds.log; exit 1; }
python3 - $O/lds <<'PY'
import csv, glob, sys, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"rollout_kernel<(\d), false, false>", r["Kernel_Name"])
        if m:
            acc[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print("policy", k, {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
