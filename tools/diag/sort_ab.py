"""A/B of the TD grouping sort (diagnostic, GPU box):
    python tools/diag/sort_ab.py LIB_ROCPRIM.so LIB_OWN.so [LIB_OWN2.so ...] [--games=N] [--reps=R]
The update words of `games` random self-play games (bench.py's td_state_map
batch: 262,144 games, ~32.2M words) sorted by both libraries' oth_td_sort_packed
and, with the build's own sort, by oth_td_sort_unpack; every output is checked
against torch's stable sort of the key bits, then each variant is timed with
HIP events (median of `reps`, 5 launches per sample, alternating)."""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib, ops  # noqa: E402
from subproc_amd.td import lam_pow_table  # noqa: E402

paths = [a for a in sys.argv[1:] if a.endswith(".so")]
opt = dict(a[2:].split("=") for a in sys.argv[1:] if a.startswith("--"))
games = int(opt.get("games", 1 << 18))
reps = int(opt.get("reps", 7))
dev = torch.device("cuda", 0)
libs = []
for p in paths:
    L = ctypes.CDLL(os.path.abspath(p))
    for name, (res, argt) in _lib.SIGNATURES.items():
        if hasattr(L, name):
            f = getattr(L, name)
            f.restype, f.argtypes = res, argt
    libs.append(L)
s = torch.cuda.current_stream().cuda_stream

r = ops.rollout(games, 0x5EED, 1 << 41, "random", record_moves=True, device=dev)
pk = ops.replay_rows(r.moves, r.plies)
cnt = 2 * (r.plies.long() + 1)
base = (torch.cumsum(cnt, 0) - cnt).contiguous()
n = int(cnt.sum())
words = torch.empty(n, dtype=torch.int64, device=dev)
assert libs[1].oth_td_updates_packed(pk.boards.data_ptr(), pk.row_off.data_ptr(), r.plies.data_ptr(), base.data_ptr(),
                                     words.data_ptr(), games, s) == 0
lam = torch.tensor(lam_pow_table(0.9), dtype=torch.float64, device=dev)
KEY = (1 << 36) - 1  # include/othello.h OTH_TD_SKEY_BITS (round 5; 43 before)
_, perm = torch.sort(words & KEY, stable=True)
want = words[perm]
print("words %d" % n, flush=True)


def scratch(fn, args):
    tb = ctypes.c_size_t(0)
    assert fn(*args, None, ctypes.byref(tb), s) == 0
    return torch.empty(max(tb.value, 1), dtype=torch.uint8, device=dev), tb


outs = []
variants = []
for tag, L in zip(["rocprim"] + [os.path.basename(p)[:-3] for p in paths[1:]], libs):
    o = torch.empty_like(words)
    t, tb = scratch(L.oth_td_sort_packed, (words.data_ptr(), o.data_ptr(), n))
    k = torch.empty_like(words)
    v = torch.empty(n, dtype=torch.float64, device=dev)
    a = (words.data_ptr(), o.data_ptr(), n, t.data_ptr(), ctypes.byref(tb), s)
    variants.append((tag + " sort_packed", L.oth_td_sort_packed, a, o, None))
    if "nolook" in tag:  # diagnostic builds whose output is unsorted by design: the sort alone
        continue
    ua = (o.data_ptr(), lam.data_ptr(), k.data_ptr(), v.data_ptr(), n, s)
    variants.append((tag + " unpack", L.oth_td_unpack, ua, None, None))
    if tag != "rocprim":
        k2 = torch.empty_like(words)
        v2 = torch.empty(n, dtype=torch.float64, device=dev)
        t2, tb2 = scratch(L.oth_td_sort_unpack, (words.data_ptr(), lam.data_ptr(), k2.data_ptr(), v2.data_ptr(), n))
        a2 = (words.data_ptr(), lam.data_ptr(), k2.data_ptr(), v2.data_ptr(), n, t2.data_ptr(), ctypes.byref(tb2), s)
        variants.append((tag + " sort_unpack", L.oth_td_sort_unpack, a2, None, (k2, v2, k, v)))
for name, fn, a, o, kv in variants:
    assert fn(*a) == 0, name
torch.cuda.synchronize()
for name, fn, a, o, kv in variants:
    if o is not None:
        print("%-20s identical to torch stable sort: %s" % (name, torch.equal(o, want)), flush=True)
    if kv is not None:
        print("%-20s keys/values identical to sort + unpack: %s" % (name, torch.equal(kv[0], kv[2]) and
                                                                    torch.equal(kv[1].view(torch.int64),
                                                                                kv[3].view(torch.int64))))
times = {v[0]: [] for v in variants}
for rep in range(reps):
    for name, fn, a, o, kv in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn(*a)
        e0.record()
        for _ in range(5):
            fn(*a)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 5)
for name, ts in times.items():
    ms = statistics.median(ts)
    print("%-20s median %.3f ms (%.3f-%.3f)  %.2f GB/s per pass-equivalent" % (name, ms, min(ts), max(ts),
                                                                              n * 16 / ms / 1e6), flush=True)
