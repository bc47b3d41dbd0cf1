"""Per-tile timeline of the build's own TD sort (diagnostic, an
OTH_SORT_ROCPRIM=0 OTH_SORT_DIAG_TIME=1 build): s_memtime at each block's
entry, before its look-back, after it, and at exit, read back from the sort's
scratch (the layout of td_table.hip's sort_plan).  python tools/diag/sort_time.py LIB.so"""
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from subproc_amd import _lib, ops  # noqa: E402

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
res, argt = _lib.SIGNATURES["oth_td_sort_packed"]
L.oth_td_sort_packed.restype, L.oth_td_sort_packed.argtypes = res, argt
s = torch.cuda.current_stream().cuda_stream
r = ops.rollout(1 << 18, 0x5EED, 1 << 41, "random", record_moves=True, device="cuda")
pk = ops.replay_rows(r.moves, r.plies)
cnt = 2 * (r.plies.long() + 1)
base = (torch.cumsum(cnt, 0) - cnt).contiguous()
n = int(cnt.sum())
w = torch.empty(n, dtype=torch.int64, device="cuda")
assert _lib.load().oth_td_updates_packed(pk.boards.data_ptr(), pk.row_off.data_ptr(), r.plies.data_ptr(),
                                         base.data_ptr(), w.data_ptr(), 1 << 18, s) == 0
o = torch.empty_like(w)
tb = ctypes.c_size_t(0)
assert L.oth_td_sort_packed(w.data_ptr(), o.data_ptr(), n, None, ctypes.byref(tb), s) == 0
t = torch.zeros(tb.value, dtype=torch.uint8, device="cuda")
for _ in range(3):
    assert L.oth_td_sort_packed(w.data_ptr(), o.data_ptr(), n, t.data_ptr(), ctypes.byref(tb), s) == 0
torch.cuda.synchronize()
al = lambda x: (x + 255) // 256 * 256  # noqa: E731
P, D, T, G = 5, 512, 4096, 16
tiles = (n + T - 1) // T
hist_off = al(8 * n)
ticket_off = al(hist_off + P * D * 8)
status_off = al(ticket_off + 9 * 4)
vec_off = (tiles + 63) // 64 * 64
gsum_off = vec_off + tiles * 2 * D
groups = (tiles + G - 1) // G
diag_off = (gsum_off + P * (groups * (D + 1) + 64) + 1) // 2 * 2
d0 = status_off + diag_off * 4
ts = t[d0: d0 + P * tiles * 32].cpu().numpy().view(np.uint64).reshape(P, tiles, 4).astype(np.int64)
for q in range(P):
    x = ts[q]
    t0 = x[:, 0].min()
    pre, look, post = x[:, 1] - x[:, 0], x[:, 2] - x[:, 1], x[:, 3] - x[:, 2]
    span = x[:, 3].max() - t0
    print("pass %d: span %d ticks; per block: before look-back %d / %d, look-back %d / %d (p90 %d, max %d), "
          "write %d / %d  (median / mean)" % (q, span, np.median(pre), pre.mean(), np.median(look), look.mean(),
                                               np.percentile(look, 90), look.max(), np.median(post), post.mean()))
    k = np.argsort(x[:, 0])
    print("   start order == tile order for %.1f%% of tiles; first-wave blocks (started before any ended): %d" % (
        100 * np.mean(k == np.arange(tiles)), int((x[:, 0] < x[:, 3].min()).sum())))
    # look-back time by tile index decile
    dec = [int(np.median(look[i * tiles // 10:(i + 1) * tiles // 10])) for i in range(10)]
    print("   look-back median by tile decile:", dec)
