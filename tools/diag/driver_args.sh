#!/bin/bash
# bench.py at the driver's arguments (--steps 20 --warmup 5) and at other K,
# to separate a fixed per-timed-region cost from the per-step time.
mkdir -p gpurun_out/drv
for k in 10 20 50 100 200; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps $k --warmup 5 > gpurun_out/drv/k$k.json 2> gpurun_out/drv/k$k.err || exit 1
done
