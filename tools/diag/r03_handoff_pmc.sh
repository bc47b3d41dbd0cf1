#!/bin/bash
# (libraries: tools/diag/build_ab_banks.sh, run here first)
# Round-3: executed VALU and busy cycles per 1M-game launch of the headline
# kernel, HEAD against the hand-over build at K = 0, 8, 16 (tools/diag/rollout_1m.py;
# warm-up launches included in the CSV, the summary takes the last 20).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/hpmc
mkdir -p $O
L=subproc_amd/lib/libsubproc_amd_hip.so
cp $L $O/libshipped.so || exit 1
for v in head new_k0 new_k8 new_k16 head2 new2_k16; do
  K=${v#*_k}; [ "$K" = "$v" ] && K=8
  case $v in new*) cp tools/diag/ab/libnew.so $L;; *) cp tools/diag/ab/libhead.so $L;; esac || exit 1
  OTH_HANDOFF_K=$K timeout -k 10 120 python3 tools/diag/rollout_1m.py > $O/$v.time.log 2>&1 || { cp $O/libshipped.so $L; cat $O/$v.time.log; exit 1; }
  OTH_HANDOFF_K=$K timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/$v -o run -- python3 tools/diag/rollout_1m.py > $O/$v.pmc.log 2>&1 || { cp $O/libshipped.so $L; tail -5 $O/$v.pmc.log; exit 1; }
  echo "$v $(cat $O/$v.time.log | grep 1M)"
done
cp $O/libshipped.so $L
python3 - <<'PY'
import csv, glob, collections
for v in ["head", "new_k0", "new_k8", "new_k16", "head2", "new2_k16"]:
    f = glob.glob("gpurun_out/hpmc/%s/**/*counter_collection.csv" % v, recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    per = collections.defaultdict(dict)
    for r in rows:
        if "rollout_kernel" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    last = [per[k] for k in sorted(per)][-20:]
    avg = {c: sum(d.get(c, 0) for d in last) / len(last) for c in last[0]}
    print(v, " ".join("%s=%.4g" % (c, x) for c, x in sorted(avg.items())))
PY
