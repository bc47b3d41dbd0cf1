#!/bin/bash
# TD spec split on the GPU box (diagnostic): its tests, the miss probe under a
# kernel trace, the split's time under each build/var/spec*.so, the TD update rate
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-tdprobe} && mkdir -p $O || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_td.py tests/test_gpu_abi_pair.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/diag/td_spec_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep -v "^W2026\|^E2026" $O/probe.log | tail -5
for v in build/var/spec*.so; do
  [ -f "$v" ] || continue
  b=$(basename $v .so)
  L=256; P=1024; case $b in spec512) L=512; P=512;; spec128) L=128; P=1024;; esac
  echo "== $b"
  SPEC_LANES=$L SPEC_PART=$P timeout -k 10 200 python3 tools/diag/td_spec_probe.py --lib=$v > $O/probe_$b.log 2>&1 || { tail -5 $O/probe_$b.log; exit 1; }
  tail -4 $O/probe_$b.log
done
timeout -k 10 200 python3 tools/diag/td_trace.py 262144 4 2>&1 | tee $O/td_product.log
for w in; do
  echo "== warm $w"
  OTH_TD_SPEC_WARM=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$w -o run -- python3 tools/diag/td_spec_probe.py > $O/probe_w$w.log 2>&1 || { tail -5 $O/probe_w$w.log; exit 1; }
  grep -v "^W2026\|^E2026" $O/probe_w$w.log | tail -4
done
