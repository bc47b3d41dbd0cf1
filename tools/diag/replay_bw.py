"""Replay-kernel traffic probe (diagnostic; run under rocprofv3 --pmc on the GPU box)."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import ops  # noqa: E402

n = 1 << 18
r = ops.rollout(n, 7, 0, "random", record_moves=True, device="cuda")
for _ in range(3):
    pos = ops.replay(r.moves, r.plies)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    pos = ops.replay(r.moves, r.plies)
e1.record()
torch.cuda.synchronize()
print("replay %d games: %.1f us/launch" % (n, e0.elapsed_time(e1) / 10 * 1e3))
