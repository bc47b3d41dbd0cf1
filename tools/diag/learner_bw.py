"""oth_features / oth_eval / oth_td_updates throughput on the recorded
positions of 262,144 random games (diagnostic, GPU box)."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import ops  # noqa: E402
from subproc_amd.params import DEFAULT_WEIGHTS  # noqa: E402

n = 1 << 18
r = ops.rollout(n, 7, 0, "random", record_moves=True, device="cuda")
pos = ops.replay(r.moves, r.plies)
boards = pos.boards.reshape(-1, 2)
m = boards.shape[0]
side = torch.randint(1, 3, (m,), dtype=torch.uint8, device="cuda")


def timeit(name, fn, nbytes):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    print("%-10s %d positions: %.1f us/launch, %.2f TB/s" % (name, m, us, nbytes / us / 1e6))


timeit("features", lambda: ops.features(boards, side), m * (16 + 1 + 10))
timeit("eval", lambda: ops.evaluate(boards, side, DEFAULT_WEIGHTS), m * (16 + 1 + 4))
