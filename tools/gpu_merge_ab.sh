#!/bin/bash
# TD merge tile A/B (diagnostic): td_trace.py under a kernel trace for each
# build/var/merge*.so (OTH_MERGE_K builds), merge and lookup kernel times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-mergeab} && mkdir -p $O || exit 1
for rep in 1 2; do
for v in build/var/merge*.so; do
  b=$(basename $v .so)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$b$rep -o run -- python3 tools/diag/td_trace.py 262144 4 --lib=$v > $O/$b$rep.log 2>&1 || { tail -5 $O/$b$rep.log; exit 1; }
  python3 - $O/$b$rep/run_kernel_stats.csv $b <<'PY'
import csv, sys
r = {x['Name'][:40]: x for x in csv.DictReader(open(sys.argv[1]))}
m = [v for k, v in r.items() if 'td_merge' in k][0]
print("%-8s merge avg %.1f us (calls %s)" % (sys.argv[2], float(m['AverageNs']) / 1e3, m['Calls']))
PY
  grep "batch 3" $O/$b$rep.log
done
done
