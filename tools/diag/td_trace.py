"""The TD state-map update of bench.py's td_state_map line, for a kernel trace
(diagnostic; run on the GPU box under rocprofv3 --kernel-trace --stats):
three 262,144-game batches of GPU self-play books into one StateMap (the empty
table, then two merges), each replayed (packed rows, as bench.py) then applied; prints the wall time
of each replay + update."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import ops  # noqa: E402
from subproc_amd.td import StateMap  # noqa: E402

args = [x for x in sys.argv[1:] if not x.startswith("--lib=")]
for x in sys.argv[1:]:
    if x.startswith("--lib="):  # an A/B build of the whole library (tools/gpu_merge_ab.sh)
        from subproc_amd import _lib
        _lib.LIB_PATH = os.path.abspath(x[len("--lib="):])
games = int(args[0]) if len(args) > 0 else 1 << 18
reps = int(args[1]) if len(args) > 1 else 3
dev = torch.device("cuda", 0)
sm = StateMap(dev)
for k in range(reps):
    r = ops.rollout(games, 0x5EED, (1 << 41) + k * games, "random", record_moves=True, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = sm.update_rows(ops.replay_rows(r.moves, r.plies), r.plies)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("batch %d: %d updates, %d keys, %.2f ms, %.3e updates/s" % (k, n, len(sm), dt * 1e3, n / dt), flush=True)
