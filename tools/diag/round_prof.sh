#!/bin/bash
# One box call: facade/engine per-ply timing, then the round profile.
# Usage (via gpurun): tools/diag/round_prof.sh r02
bash tools/diag/facade_check.sh || exit 1
bash tools/profile_round.sh "$1" || exit 1
