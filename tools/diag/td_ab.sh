#!/bin/bash
# TD A/B (diagnostic, round 5): tools/diag/td_trace.py under a kernel trace
# for each build/var/<name>.so given (two passes), the TD kernels' average
# times and the batch wall times.   usage: td_ab.sh OUTDIR name1 name2 ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/$1 && shift && mkdir -p $O || exit 1
for rep in 1 2; do
for b in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$b$rep -o run -- python3 tools/diag/td_trace.py 262144 4 --lib=build/var/$b.so > $O/$b$rep.log 2>&1 || { tail -5 $O/$b$rep.log; exit 1; }
  python3 - $O/$b$rep/run_kernel_stats.csv $b <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0.0
for x in rows:
    nm = x['Name']
    if 'rollout' in nm:
        continue
    tot += float(x['TotalDurationNs'])
    if any(k in nm for k in ('td_merge', 'td_lookup', 'td_splits', 'td_seg_kernel', 'td_updates', 'td_ema', 'replay')):
        print("%-12s %-44s avg %8.1f us calls %s" % (sys.argv[2], nm[:44], float(x['AverageNs']) / 1e3, x['Calls']))
print("%-12s kernels other than the rollout: %.3f ms per batch (4 batches)" % (sys.argv[2], tot / 4e6))
PY
  grep "batch 3" $O/$b$rep.log
done
done
