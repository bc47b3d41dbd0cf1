#!/bin/bash
# TD EMA fork A/B (diagnostic, round 5): tools/diag/td_trace.py on the in-tree
# library with OTH_TD_EMA_FORK=0 (every EMA kernel on the caller's stream) and
# =1 (long and split keys on side streams; 1p: at normal priority,
# OTH_TD_EMA_PRIO=0), alternating, three passes; then one
# kernel trace of each for the batch timeline (tools/diag/td_gaps.py).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-tdfork} && mkdir -p $O || exit 1
for rep in 1 2 3; do
  for f in 0 1 1p; do
    [ $f = 1p ] && export OTH_TD_EMA_PRIO=0 || export OTH_TD_EMA_PRIO=1
    OTH_TD_EMA_FORK=${f:0:1} timeout -k 10 200 python3 tools/diag/td_trace.py 262144 4 > $O/f$f.$rep.log 2>&1 || { tail -5 $O/f$f.$rep.log; exit 1; }
    echo "fork=$f pass $rep: $(grep -E '^batch [23]' $O/f$f.$rep.log | tr '\n' ' ')"
  done
done
export OTH_TD_EMA_PRIO=1
for f in 0 1; do
  OTH_TD_EMA_FORK=$f timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr$f -o run -- python3 tools/diag/td_trace.py 262144 4 > $O/tr$f.log 2>&1 || { tail -5 $O/tr$f.log; exit 1; }
  python3 tools/diag/td_gaps.py $(find $O/tr$f -name '*kernel_trace.csv') > $O/gaps$f.txt && tail -1 $O/gaps$f.txt
done
