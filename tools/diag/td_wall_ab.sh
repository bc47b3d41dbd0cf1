#!/bin/bash
# TD batch wall-time A/B (diagnostic, round 5): tools/diag/td_trace.py (4
# batches of 262,144 random games) for each build/var/<name>.so given,
# alternating, three passes, without a profiler; then one kernel trace of each
# for its batch timeline (tools/diag/td_gaps.py).   usage: td_wall_ab.sh OUTDIR name1 name2 ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/$1 && shift && mkdir -p $O || exit 1
for rep in 1 2 3; do
  for b in "$@"; do
    timeout -k 10 200 python3 tools/diag/td_trace.py 262144 4 --lib=build/var/$b.so > $O/$b.$rep.log 2>&1 || { tail -5 $O/$b.$rep.log; exit 1; }
    echo "$b pass $rep: $(grep -E '^batch [23]' $O/$b.$rep.log | sed 's/ updates, [0-9]* keys//' | tr '\n' ' ')"
  done
done
for b in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$b -o run -- python3 tools/diag/td_trace.py 262144 4 --lib=build/var/$b.so > $O/tr_$b.log 2>&1 || { tail -5 $O/tr_$b.log; exit 1; }
  python3 tools/diag/td_gaps.py $(find $O/tr_$b -name '*kernel_trace.csv') > $O/gaps_$b.txt && echo "$b $(tail -1 $O/gaps_$b.txt)"
done
