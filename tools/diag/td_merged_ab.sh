mkdir -p gpurun_out/mg2 && timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_td.py > gpurun_out/mg2/t.log 2>&1; rc=$?; tail -1 gpurun_out/mg2/t.log; [ $rc = 0 ] || exit 1
for rep in 1 2 3; do for m in 1 0; do OTH_TD_EMA_MERGED=$m timeout -k 10 120 python3 tools/diag/td_bench_ab.py build/var/cur.so > gpurun_out/mg2/s$m$rep.log 2>&1 || exit 1; echo "merged=$m $(tail -1 gpurun_out/mg2/s$m$rep.log)"; done; done
OTH_TD_EMA_MERGED=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mg2/tr -o run -- python3 tools/diag/td_trace.py 262144 4 --lib=build/var/cur.so > gpurun_out/mg2/tr.log 2>&1 || exit 1
python3 tools/diag/td_gaps.py $(find gpurun_out/mg2/tr -name '*kernel_trace.csv') | tail -12
