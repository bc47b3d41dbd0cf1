"""oth_book_text throughput (diagnostic, GPU box): serialize_str text of the
16M recorded positions of 262,144 random games (~1.07 GB of text)."""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import ops  # noqa: E402

n = 1 << 18
r = ops.rollout(n, 7, 0, "random", record_moves=True, device="cuda")
pos = ops.replay(r.moves, r.plies)
boards = pos.boards.reshape(-1, 2)
turn = pos.turn.reshape(-1)
m = boards.shape[0]
for _ in range(3):
    txt = ops.book_text(boards, turn)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    txt = ops.book_text(boards, turn)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 10 * 1e3
nbytes = m * 67 + m * 17
print("book_text %d positions: %.1f us/launch, %.2f TB/s (67 B written + 17 B read per position)" % (m, us,
                                                                                                    nbytes / us / 1e6))
