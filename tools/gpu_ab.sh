#!/bin/bash
# same-box A/B runs of round-4 variants (diagnostic): the 1-ply choice builds,
# a kernel trace of the TD state-map update, and the TD update under the sort
# digit-width builds (each present build/var/*.so is used)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
COOP=$(ls build/var/r03coop.so build/var/keep0.so build/var/cur.so 2>/dev/null)
if [ -n "$COOP" ]; then
  timeout -k 10 400 python tools/diag/policy_ab.py $COOP --policies greedy,eval --reps 5 > $O/coop_ab.log 2>&1 || { cat $O/coop_ab.log; exit 1; }
  cat $O/coop_ab.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/td -o run -- python3 tools/diag/td_trace.py > $O/td_trace.log 2>&1 || { tail -5 $O/td_trace.log; exit 1; }
grep batch $O/td_trace.log
for v in build/var/sort*.so; do
  [ -f "$v" ] || continue
  echo "== $v"
  timeout -k 10 200 python3 tools/diag/td_trace.py 262144 4 --lib=$v > $O/td_$(basename $v .so).log 2>&1 || { tail -5 $O/td_$(basename $v .so).log; exit 1; }
  cat $O/td_$(basename $v .so).log
done
echo "== product"
timeout -k 10 200 python3 tools/diag/td_trace.py 262144 4 2>&1 | tee $O/td_product.log
