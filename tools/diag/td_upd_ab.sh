#!/bin/bash
# TD update-stream kernel A/B (diagnostic, round 5): td_trace.py under a kernel
# trace for build/var/skey.so (+ the 36-bit sort key), upd_wave.so (one wave per game, 43-bit key) and upd_slot.so
# (OTH_TD_UPD_WAVE=0, one thread per 129-row slot); the update kernel's time
# and the batch wall times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-updab} && mkdir -p $O || exit 1
for rep in 1 2; do
for b in skey upd_wave; do
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
    if 'td_updates' in nm or 'td_seg' in nm or 'onesweep' in nm or 'histogram' in nm:
        print("%-9s %-60s avg %8.1f us calls %s" % (sys.argv[2], nm[:60], float(x['AverageNs']) / 1e3, x['Calls']))
print("%-9s kernels other than the rollout: %.3f ms per batch (4 batches)" % (sys.argv[2], tot / 4e6))
PY
  grep "batch 3" $O/$b$rep.log
done
done
