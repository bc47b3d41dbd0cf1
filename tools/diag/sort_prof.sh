#!/bin/bash
# sort_ab.py under a kernel trace (diagnostic): per-kernel average times of the
# TD sort variants.  Usage (GPU box): tools/diag/sort_prof.sh OUT LIB.so ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python tools/diag/sort_ab.py "$@" --reps=5 > $O/ab.log 2>&1 || { tail -5 $O/ab.log; exit 1; }
grep -v unpack $O/ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/diag/sort_ab.py "$@" --reps=2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("sort_", "rocprim", "td_unpack", "fillBuffer")):
        print("%-70s %6s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
