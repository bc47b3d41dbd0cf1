mkdir -p gpurun_out/drv
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv/s20_$i.json 2> gpurun_out/drv/s20_$i.err || exit 1; done
timeout -k 10 300 python3 bench.py > gpurun_out/drv/def.json 2> gpurun_out/drv/def.err || exit 1
