#!/bin/bash
# Step-kernel A/B on the GPU box: timing with and without legal_next, then a
# VALU/VMEM PMC pass, for each library in $LIBS (diagnostic builds of kernel
# variants exposing the same C-ABI; default: the product library).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sv
LIBS="${LIBS:-subproc_amd/lib/libsubproc_amd_hip.so}"
for L in $LIBS; do
  timeout -k 10 120 python tools/diag/step_sweep.py "$L" || exit 1
  timeout -k 10 120 python tools/diag/step_sweep.py "$L" --no-legal || exit 1
done
for L in $LIBS; do
  b=$(basename "$L" .so)
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d gpurun_out/sv/pmc_$b -o run -- python3 tools/diag/step_sweep.py "$L" > gpurun_out/sv/pmc_$b.log 2>&1 || exit 1
  echo "== $b"; python3 tools/pmc_summary.py --match=step gpurun_out/sv/pmc_$b/run_counter_collection.csv
done
