"""Time oth_td_ema_split of two library builds on one batch's update stream (GPU box).
  python tools/diag/td_ema_ab.py LIB_A.so LIB_B.so"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib, ops, td  # noqa: E402

dev = torch.device("cuda", 0)
r = ops.rollout(1 << 18, 0x5EED, 1 << 41, "random", record_moves=True, device=dev)
pos = ops.replay(r.moves, r.plies)
plies = r.plies
cnt = 2 * (plies.long() + 1)
ends = torch.cumsum(cnt, 0)
base = ends - cnt
total = int(ends[-1])
keys = torch.empty(total, dtype=torch.int64, device=dev)
vals = torch.empty(total, dtype=torch.float64, device=dev)
lib0 = _lib.load()
st = torch.cuda.current_stream().cuda_stream
lam = torch.tensor(td.lam_pow_table(), dtype=torch.float64, device=dev)
_lib.check(lib0.oth_td_updates(pos.boards.data_ptr(), plies.data_ptr(), base.data_ptr(), lam.data_ptr(),
                               keys.data_ptr(), vals.data_ptr(), plies.numel(), st), "u")
sk, perm = torch.sort(keys, stable=True)
sv = vals[perm].contiguous()
uk, counts = torch.unique_consecutive(sk, return_counts=True)
seg = torch.zeros(uk.numel() + 1, dtype=torch.int64, device=dev)
torch.cumsum(counts, 0, out=seg[1:])
init = torch.zeros(uk.numel(), dtype=torch.float64, device=dev)
LONG_MIN = int(os.environ.get("TD_LONG_MIN", td.LONG_MIN))
li = torch.nonzero(counts >= LONG_MIN).flatten()
print("long_min", LONG_MIN, "long segments", li.numel())
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    L.oth_td_ema_split.restype, L.oth_td_ema_split.argtypes = _lib.SIGNATURES["oth_td_ema_split"]
    out = torch.empty_like(init)
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        L.oth_td_ema_split(sv.data_ptr(), seg.data_ptr(), init.data_ptr(), 0.03, 0.97, out.data_ptr(), uk.numel(),
                           LONG_MIN, li.data_ptr(), li.numel(), st)
        torch.cuda.synchronize()
        print("%-24s %.2f ms" % (os.path.basename(path), (time.perf_counter() - t) * 1e3))
