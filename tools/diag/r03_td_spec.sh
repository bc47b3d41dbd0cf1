#!/bin/bash
# Round 3: the TD EMA speculation kernel with its parts' values staged through
# LDS (coalesced loads) and two chains per lane -- TD tests, then a kernel
# trace of tools/diag/td_stages.py and the bench's TD line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/tdspec
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_td.py tests/test_gpu_ingest.py tests/test_gpu_abi_pair.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/diag/td_stages.py > $O/td_stages.log 2>&1 || { tail -20 $O/td_stages.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/tdspec/kt/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'td_' in r['Name']:
        print("%8.1f us x%s  %s" % (float(r['AverageNs']) / 1e3, r['Calls'], r['Name'][:60]))
PY
