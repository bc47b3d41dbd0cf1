#!/bin/bash
# same-box A/B runs of round-4 variants (diagnostic): the 1-ply choice builds,
# the step builds (if present), and a kernel trace of the TD state-map update
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
if [ -f build/var/pipe.so ]; then
  timeout -k 10 400 python tools/diag/policy_ab.py build/var/r03coop.so build/var/pipe.so build/var/nopipe.so build/var/keep0.so --policies greedy,eval --reps 5 > $O/coop_ab.log 2>&1 || { cat $O/coop_ab.log; exit 1; }
  cat $O/coop_ab.log
fi
if [ -f build/var/step_k1.so ]; then
  timeout -k 10 200 python tools/diag/step_ab.py build/var/step_k1.so build/var/step_k2.so 5 > $O/step_ab.log 2>&1 || { cat $O/step_ab.log; exit 1; }
  tail -4 $O/step_ab.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/td -o run -- python3 tools/diag/td_trace.py > $O/td_trace.log 2>&1 || { tail -5 $O/td_trace.log; exit 1; }
cat $O/td_trace.log
