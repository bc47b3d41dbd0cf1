#!/bin/bash
# Round 3: the random policy's move records built in LDS and written per wave
# (rollout_kernel<0, true>) -- every test that records moves, then the round
# profile for the record kernel's HBM traffic.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/recstage
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
./tools/profile_round.sh r03 > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo profiled
