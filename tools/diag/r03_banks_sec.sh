#!/bin/bash
# (libraries: tools/diag/build_ab_banks.sh, run here first)
# Round-3: the VGPR-bank pass on the secondary kernels (greedy, eval, step,
# TD, replay): the full bench line, two passes over HEAD, HEAD + bank pass and
# the in-tree library.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/banks_sec
mkdir -p $O
L=subproc_amd/lib/libsubproc_amd_hip.so
cp $L $O/libshipped.so || exit 1
export BENCH_SKIP=rollout_16M
for pass in 1 2; do
  for v in head head_bank new; do
    case $v in new) cp tools/diag/ab/libnew.so $L;; *) cp tools/diag/ab/lib$v.so $L;; esac || exit 1
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/$v.$pass.json 2> $O/$v.$pass.err || { cp $O/libshipped.so $L; tail -5 $O/$v.$pass.err; exit 1; }
    tail -1 $O/$v.$pass.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['secondary']
def g(k, f='value'):
    x=s.get(k,{}); return x.get(f) if isinstance(x,dict) else None
print('%-9s head %.4g  greedy %.4g  eval %.4g  step65k %.4g  step16M %.4g  1stream %.4g' % (sys.argv[1], d['value'], g('greedy_1M'), g('eval_1M'), g('step_65536'), g('step_steady_16M'), g('rollout_1stream')))
print('   td', json.dumps(s.get('td_state_map'))[:400])
print('   books', json.dumps(s.get('book_emitter'))[:600])
" $v
  done
done
cp $O/libshipped.so $L
