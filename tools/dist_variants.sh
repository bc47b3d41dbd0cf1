#!/bin/bash
# RCCL histogram all-reduce placement at world size 1 (torchrun), vs plain N=1.
set -o pipefail
mkdir -p gpurun_out/dv
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-secondary > gpurun_out/dv/plain_$i.log 2>&1 || exit 1
  for v in async sync end; do
    BENCH_FORCE_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2954$i bench.py --gpus 1 --steps 20 --warmup 3 --no-secondary --allreduce $v > gpurun_out/dv/${v}_$i.log 2>&1 || exit 1
  done
done
for f in gpurun_out/dv/*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e9,2), "Gsteps/s", round(d["ms_per_step"],4), "ms")')"; done
