#!/bin/bash
# Hand-over K on one box (round 6): the config-3 bench line at the driver's
# arguments for K = 8, 12, 16 (three passes, alternating), then per K one
# WRITE_SIZE and one FETCH_SIZE pass over three 1M-game random launches.
# Usage (GPU box): [KS="8 12 16"] [REPS=3] tools/gpu_handoff_k.sh OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
mkdir -p $O
for rep in $(seq ${REPS:-3}); do
  for k in ${KS:-8 12 16}; do
    OTH_HANDOFF_K=$k timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-secondary > $O/k${k}_$rep.log 2>&1 || { tail -5 $O/k${k}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print('K=%-3s %.4e  %.4f ms/step' % (sys.argv[2], d['value'], d['ms_per_step']))" $O/k${k}_$rep.log $k | tee -a $O/k.txt
  done
done
for k in ${KS:-8 12 16}; do
  for c in WRITE_SIZE FETCH_SIZE; do
    OTH_HANDOFF_K=$k timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${k}_$c -o run -- python3 tools/diag/lds_probe.py random > $O/pmc_${k}_$c.log 2>&1 || { tail -5 $O/pmc_${k}_$c.log; exit 1; }
  done
done
KS="${KS:-8 12 16}" python3 - $O <<'PY'
import csv, glob, sys, re, collections
import os
for k in map(int, os.environ["KS"].split()):
    out = {}
    for c in ("WRITE_SIZE", "FETCH_SIZE"):
        v = []
        for f in glob.glob("%s/pmc_%d_%s/**/*counter_collection.csv" % (sys.argv[1], k, c), recursive=True):
            for r in csv.DictReader(open(f)):
                if re.search(r"rollout_kernel<0, false, false>", r["Kernel_Name"]) and r["Counter_Name"] == c:
                    v.append(float(r["Counter_Value"]))
        out[c] = sum(v) / len(v) * 1024 if v else None
    hbm = out["WRITE_SIZE"] + 2 * out["FETCH_SIZE"]
    print("K=%d write %.3f MB fetch(x2) %.3f MB total %.3f MB = %.3fx the 18.874 MB algorithmic" % (
        k, out["WRITE_SIZE"] / 1e6, 2 * out["FETCH_SIZE"] / 1e6, hbm / 1e6, hbm / 18874368))
PY
