"""The build's own TD sort on growing sizes (diagnostic, GPU box): output
against torch's stable sort of the key bits, and the sort's look-back error
word (bits: 1 a tile word never seen, 2 phase-A poll, 4 phase-B poll, 8 walk
ran past group 0).  python tools/diag/sort_small.py LIB.so [sizes...]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib  # noqa: E402

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
res, argt = _lib.SIGNATURES["oth_td_sort_packed"]
L.oth_td_sort_packed.restype, L.oth_td_sort_packed.argtypes = res, argt
td = "--td" in sys.argv  # the TD update words of 262,144 random games (skewed keys), as sort_ab.py
sizes = [int(x) for x in sys.argv[2:] if not x.startswith("--")] or [1000, 100_000, 1_000_000, 8_000_000, 32_000_000]
s = torch.cuda.current_stream().cuda_stream
g = torch.Generator(device="cuda").manual_seed(1)
KEY = (1 << 36) - 1  # include/othello.h OTH_TD_SKEY_BITS (round 5; 43 before)
if td:
    from subproc_amd import ops
    r = ops.rollout(1 << 18, 0x5EED, 1 << 41, "random", record_moves=True, device="cuda")
    pk = ops.replay_rows(r.moves, r.plies)
    cnt = 2 * (r.plies.long() + 1)
    base = (torch.cumsum(cnt, 0) - cnt).contiguous()
    W = torch.empty(int(cnt.sum()), dtype=torch.int64, device="cuda")
    assert _lib.load().oth_td_updates_packed(pk.boards.data_ptr(), pk.row_off.data_ptr(), r.plies.data_ptr(),
                                             base.data_ptr(), W.data_ptr(), 1 << 18, s) == 0
    sizes = [n for n in sizes if n <= W.numel()] + [W.numel()]
for n in sizes:
    if td:
        w = W[:n].contiguous()
    else:
        k = torch.randint(0, 1 << 20, (n,), device="cuda", generator=g) * 8388593 & KEY
        w = k | (torch.arange(n, device="cuda") << 36)
    o = torch.empty_like(w)
    tb = ctypes.c_size_t(0)
    assert L.oth_td_sort_packed(w.data_ptr(), o.data_ptr(), n, None, ctypes.byref(tb), s) == 0
    t = torch.zeros(tb.value, dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    assert L.oth_td_sort_packed(w.data_ptr(), o.data_ptr(), n, t.data_ptr(), ctypes.byref(tb), s) == 0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    al = lambda x: (x + 255) // 256 * 256  # noqa: E731  (sort_plan's layout)
    ticket_off = al(al(8 * n) + 5 * 512 * 8)
    err = int(t[ticket_off + 32: ticket_off + 36].cpu().view(torch.int32)[0])
    _, perm = torch.sort(w & KEY, stable=True)
    print("n %d: %.3f ms, identical %s, error word %d" % (n, dt * 1e3, torch.equal(o, w[perm]), err), flush=True)
