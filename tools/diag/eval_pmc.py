"""One library's 1-ply-policy rollouts for a PMC pass (diagnostic, GPU box):
3 launches of 1,048,576 games from the opening, 10 random plies, one stream;
eval (the learner's default weights) or, with --greedy, greedy.  --children:
also count the children the 1-ply choice evaluates (every legal move of every
position from ply 10 on where the mover has a move; and without the positions
with exactly one legal move, which OTH_COOP_FORCED=1 builds play unscored),
from the move records replayed.
    rocprofv3 --pmc ... -- python3 tools/diag/eval_pmc.py LIB.so [--greedy]"""
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib  # noqa: E402
from subproc_amd.ops import _weights_ptr  # noqa: E402
from subproc_amd.params import DEFAULT_WEIGHTS  # noqa: E402

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
for name in ("oth_rollout", "oth_rollout_eval"):
    res, argt = _lib.SIGNATURES[name]
    getattr(L, name).restype, getattr(L, name).argtypes = res, argt
greedy = "--greedy" in sys.argv
n = 1 << 20
dev = torch.device("cuda", 0)
fb = torch.empty((n, 2), dtype=torch.int64, device=dev)
df = torch.empty(n, dtype=torch.int8, device=dev)
pl = torch.empty(n, dtype=torch.uint8, device=dev)
h = torch.zeros(133, dtype=torch.int64, device=dev)
wk = torch.zeros(1, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
wp = _weights_ptr(DEFAULT_WEIGHTS)
for k in range(3):
    if greedy:
        rc = L.oth_rollout(None, None, 0x5EED, k * n, 1, 10, fb.data_ptr(), df.data_ptr(), pl.data_ptr(), None,
                           h.data_ptr(), wk.data_ptr(), n, s)
    else:
        rc = L.oth_rollout_eval(None, None, 0x5EED, k * n, 10, wp, fb.data_ptr(), df.data_ptr(), pl.data_ptr(), None,
                                h.data_ptr(), wk.data_ptr(), n, s)
    assert rc == 0, rc
torch.cuda.synchronize()
print("env-steps %d" % int(h[132]))
if "--children" in sys.argv:
    from subproc_amd import ops
    m = 1 << 18
    if greedy:
        r = ops.rollout(m, 0x5EED, 0, "greedy", 10, record_moves=True, device=dev)
    else:
        r = ops.rollout(m, 0x5EED, 0, "eval", 10, record_moves=True, weights=DEFAULT_WEIGHTS, device=dev)
    rp = ops.replay(r.moves, r.plies)
    p = torch.arange(129, device=dev)[None, :]
    live = (p >= 10) & (p < r.plies.long()[:, None])
    leg = ops.legal(rp.boards.view(-1, 2), rp.turn.view(-1)).view(m, 129)
    cnt = torch.zeros_like(leg)
    x = leg.clone()
    for _ in range(64):  # popcount of the int64 masks
        cnt += x & 1
        x = (x >> 1) & 0x7FFFFFFFFFFFFFFF
    c = (cnt * live).sum().item()
    c2 = (cnt * live * (cnt >= 2)).sum().item()
    one = (live & (cnt == 1)).sum().item()
    print("children per game %.3f, %.3f at positions with >= 2 moves; %.3f positions a game with one move, "
          "%.3f choosing (%d games), plies per game %.3f" % (c / m, c2 / m, one / m, (live & (cnt >= 1)).sum().item() / m,
                                                            m, r.plies.float().mean().item()))
