#!/bin/bash
# headline stream/occupancy A/B on one box (diagnostic): bench.py's rollout
# line at the driver's --steps 20 --warmup 5 under stream counts and blocks/CU
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-streams} && mkdir -p $O || exit 1
for rep in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-secondary --streams 2 > $O/s2_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=[json.loads(l) for l in open('$O/s2_$rep.log') if l.startswith('{')][-1]; print('s2 bpc3   %.4e  %.4f ms' % (d['value'], d['ms_per_step']))"
  timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-secondary --streams 3 > $O/s3_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=[json.loads(l) for l in open('$O/s3_$rep.log') if l.startswith('{')][-1]; print('s3 bpc3   %.4e  %.4f ms' % (d['value'], d['ms_per_step']))"
  OTH_ROLLOUT_BLOCKS_PER_CU=2 timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-secondary --streams 3 > $O/s3b2_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=[json.loads(l) for l in open('$O/s3b2_$rep.log') if l.startswith('{')][-1]; print('s3 bpc2   %.4e  %.4f ms' % (d['value'], d['ms_per_step']))"
  OTH_ROLLOUT_BLOCKS_PER_CU=2 timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-secondary --streams 4 > $O/s4b2_$rep.log 2>&1 || exit 1
  python3 -c "import json; d=[json.loads(l) for l in open('$O/s4b2_$rep.log') if l.startswith('{')][-1]; print('s4 bpc2   %.4e  %.4f ms' % (d['value'], d['ms_per_step']))"
done
