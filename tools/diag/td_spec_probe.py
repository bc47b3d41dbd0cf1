"""Speculation misses of the TD spec split (diagnostic; run on the GPU box):
one 262,144-game batch into an empty StateMap, then a second batch whose
key-sorted update stream is captured; for every key of >= 4 * warm updates
the parts' warm-up guesses are replayed on the host with the exact rule (the
same part geometry as td_spec_key) and compared with the sequential state at
each part's start.  Prints keys, parts and misses, and the time of the
oth_td_ema_split launch alone over the captured stream."""
import math
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from subproc_amd import ops, td  # noqa: E402
from subproc_amd._lib import load  # noqa: E402

args = [x for x in sys.argv[1:] if not x.startswith("--lib=")]
for x in sys.argv[1:]:
    if x.startswith("--lib="):  # an A/B build of the whole library
        from subproc_amd import _lib
        _lib.LIB_PATH = os.path.abspath(x[len("--lib="):])
games = int(args[0]) if args else 1 << 18
dev = torch.device("cuda", 0)
sm = td.StateMap(dev)
cap = {}
orig = sm._apply_sorted


def grab(sk, sv):
    cap["sk"], cap["sv"] = sk.clone(), sv.clone()
    cap["keys_before"], cap["vals_before"] = sm.keys.clone() if len(sm) else None, sm.values.clone() if len(sm) else None
    orig(sk, sv)


sm._apply_sorted = grab
for k in range(2):
    r = ops.rollout(games, 0x5EED, (1 << 41) + k * games, "random", record_moves=True, device=dev)
    sm.update(ops.replay(r.moves, r.plies).boards, r.plies)
torch.cuda.synchronize()
a, oma = sm.a, 1 - sm.a
warm = int(os.environ.get("OTH_TD_SPEC_WARM", 0)) or math.ceil(-64 * math.log(2) / math.log(abs(oma)) * 4 / 3)
warm16 = (warm + 15) // 16 * 16
sk, sv = cap["sk"], cap["sv"]
ukeys, counts = torch.unique_consecutive(sk, return_counts=True)
seg = torch.zeros(ukeys.numel() + 1, dtype=torch.int64, device=dev)
torch.cumsum(counts, 0, out=seg[1:])
# state before the batch
kb, vb = cap["keys_before"], cap["vals_before"]
pos = torch.searchsorted(kb, ukeys).clamp(max=kb.numel() - 1)
init = torch.where(kb[pos] == ukeys, vb[pos], torch.zeros_like(vb[pos]))
spec = torch.nonzero(counts >= 4 * warm).flatten().tolist()
print("warm", warm, "spec keys", len(spec), "long keys", int((counts >= td.LONG_MIN).sum()), flush=True)


def run(v, xs):
    for x in xs:
        v = x if v == 0.0 else v * oma + x * a
    return v


tot_miss = 0
segh = seg.cpu().numpy()
svh = sv.cpu().numpy()
inith = init.cpu().numpy()
for s in spec[:40]:
    b, e = int(segh[s]), int(segh[s + 1])
    n = e - b
    ln = 1040  # kSpecLen
    parts = (n + ln - 1) // ln
    x = svh[b:e].tolist()
    v = float(inith[s])
    miss = 0
    for p in range(parts):
        i = p * ln
        ws = max(0, i - warm16)
        g = run(float(inith[s]) if ws == 0 else 0.0, x[ws:i])
        if g != v:
            miss += 1
        v = run(v, x[i:min(i + ln, n)])
    tot_miss += miss
    print("key %d: n %d parts %d len %d misses %d" % (s, n, parts, ln, miss), flush=True)
print("total misses (first 40 spec keys):", tot_miss, flush=True)
# the split launch alone, over the captured stream
long_idx = torch.nonzero(counts >= td.LONG_MIN).flatten()
out = torch.empty_like(init)
lib = load()
st = torch.cuda.current_stream()
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    td._with_scratch(lib.oth_td_ema_split, (sv.data_ptr(), seg.data_ptr(), init.data_ptr(), a, oma, out.data_ptr(),
                                            ukeys.numel(), td.LONG_MIN, long_idx.data_ptr(), long_idx.numel(),
                                            sv.numel()), st.cuda_stream, dev, "oth_td_ema_split")
    rc = 0
    e1.record(st)
    torch.cuda.synchronize()
    print("oth_td_ema_split rc %d: %.1f us" % (rc, e0.elapsed_time(e1) * 1e3), flush=True)
