"""Stage timing of StateMap.update (diagnostic; run on the GPU box)."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib, ops, td  # noqa: E402

dev = torch.device("cuda", 0)
games = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
r = ops.rollout(games, 0x5EED, 1 << 41, "random", record_moves=True, device=dev)
r2 = ops.rollout(games, 0x5EED, (1 << 41) + games, "random", record_moves=True, device=dev)
sm = td.StateMap(dev)
r0 = ops.rollout(games, 0x5EED, (1 << 41) + 2 * games, "random", record_moves=True, device=dev)
sm.update(ops.replay(r0.moves, r0.plies).boards, r0.plies)
sm.update(ops.replay(r.moves, r.plies).boards, r.plies)  # new keys: warms the merge path (first-use loading)
torch.cuda.synchronize()

T = {}


def mark(name, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    T[name] = T.get(name, 0) + (t - t0) * 1e3
    return t


t = time.perf_counter()
pos = ops.replay(r2.moves, r2.plies)
t = mark("replay", t)
plies = r2.plies
n = plies.shape[0]
cnt = 2 * (plies.long() + 1)
ends = torch.cumsum(cnt, 0)
base = ends - cnt
total = int(ends[-1])
keys = torch.empty(total, dtype=torch.int64, device=dev)
vals = torch.empty(total, dtype=torch.float64, device=dev)
t = mark("alloc+scan", t)
lib = _lib.load()
st = torch.cuda.current_stream().cuda_stream
_lib.check(lib.oth_td_updates(pos.boards.data_ptr(), plies.data_ptr(), base.data_ptr(), sm._lam_pow.data_ptr(),
                              keys.data_ptr(), vals.data_ptr(), n, st), "u")
t = mark("td_updates", t)
sk, perm = torch.sort(keys, stable=True)
t = mark("sort", t)
sv = vals[perm].contiguous()
t = mark("gather", t)
import ctypes  # noqa: E402
lib = _lib.load()
st = torch.cuda.current_stream().cuda_stream
sk2, sv2 = torch.empty_like(keys), torch.empty_like(vals)
tb = ctypes.c_size_t(0)
_lib.check(lib.oth_td_sort_pairs(keys.data_ptr(), vals.data_ptr(), sk2.data_ptr(), sv2.data_ptr(), total, None,
                                 ctypes.byref(tb), st), "q")
temp = torch.empty(tb.value, dtype=torch.uint8, device=dev)
t = mark("sort_pairs_alloc", t)
_lib.check(lib.oth_td_sort_pairs(keys.data_ptr(), vals.data_ptr(), sk2.data_ptr(), sv2.data_ptr(), total,
                                 temp.data_ptr(), ctypes.byref(tb), st), "s")
t = mark("sort_pairs", t)
assert torch.equal(sk, sk2) and torch.equal(sv, sv2)
t = time.perf_counter()
ukeys, counts = torch.unique_consecutive(sk, return_counts=True)
t = mark("unique", t)
seg_off = torch.zeros(ukeys.numel() + 1, dtype=torch.int64, device=dev)
torch.cumsum(counts, 0, out=seg_off[1:])
init = torch.zeros(ukeys.numel(), dtype=torch.float64, device=dev)
pos_in_old = torch.searchsorted(sm.keys, ukeys)
cl = pos_in_old.clamp(max=len(sm) - 1)
init = torch.where(sm.keys[cl] == ukeys, sm.values[cl], init)
t = mark("lookup", t)
out = torch.empty_like(init)
_lib.check(lib.oth_td_ema(sv.data_ptr(), seg_off.data_ptr(), init.data_ptr(), 0.03, 0.97, out.data_ptr(),
                          ukeys.numel(), st), "e")
t = mark("td_ema", t)
long_idx = torch.nonzero(counts >= td.LONG_MIN).flatten()
t = mark("long_idx", t)
out2 = torch.empty_like(init)
_lib.check(lib.oth_td_ema_split(sv.data_ptr(), seg_off.data_ptr(), init.data_ptr(), 0.03, 0.97, out2.data_ptr(),
                                ukeys.numel(), td.LONG_MIN, long_idx.data_ptr(), long_idx.numel(), st), "s")
t = mark("td_ema_split", t)
assert torch.equal(out, out2)
print("long segments", long_idx.numel())
print("max segment", int(counts.max()), "segments", ukeys.numel(), "updates", total)
torch.cuda.synchronize()
t = time.perf_counter()  # (the check and the prints above are not a stage)
n_old, n_upd = len(sm), ukeys.numel()
rank_in_upd = torch.searchsorted(ukeys, sm.keys)
t = mark("m.ss_old_in_upd", t)
cl = rank_in_upd.clamp(max=n_upd - 1)
hit = ukeys[cl] == sm.keys
t = mark("m.hit", t)
new_before = torch.zeros(n_upd + 1, dtype=torch.int64, device=dev)
torch.cumsum((sm.keys[pos_in_old.clamp(max=n_old - 1)] != ukeys).long(), 0, out=new_before[1:])
n_new = int(new_before[-1])
t = mark("m.cumsum", t)
old_vals = torch.where(hit, out[cl], sm.values)
pos_old = torch.arange(n_old, device=dev) + new_before[rank_in_upd]
pos_upd = new_before[:-1] + pos_in_old
t = mark("m.pos", t)
keys = torch.empty(n_old + n_new, dtype=torch.int64, device=dev)
vals = torch.empty(n_old + n_new, dtype=torch.float64, device=dev)
t = mark("m.alloc", t)
keys[pos_old] = sm.keys
vals[pos_old] = old_vals
keys[pos_upd] = ukeys
vals[pos_upd] = out
t = mark("m.scatter", t)
hit_u = sm.keys[pos_in_old.clamp(max=n_old - 1)] == ukeys
nb2 = torch.zeros(n_upd + 1, dtype=torch.int64, device=dev)
torch.cumsum(~hit_u, 0, out=nb2[1:])
t = mark("k.cumsum", t)
k2 = torch.empty(n_old + n_new, dtype=torch.int64, device=dev)
v2 = torch.empty(n_old + n_new, dtype=torch.float64, device=dev)
t = mark("k.alloc", t)
_lib.check(lib.oth_td_merge(sm.keys.data_ptr(), sm.values.data_ptr(), n_old, ukeys.data_ptr(), out.data_ptr(),
                            nb2.data_ptr(), n_upd, k2.data_ptr(), v2.data_ptr(), st), "m")
t = mark("k.merge", t)
init2 = torch.empty(n_upd, dtype=torch.float64, device=dev)
isn = torch.empty(n_upd, dtype=torch.uint8, device=dev)
t = time.perf_counter()
_lib.check(lib.oth_td_lookup(sm.keys.data_ptr(), sm.values.data_ptr(), n_old, ukeys.data_ptr(), n_upd,
                             init2.data_ptr(), isn.data_ptr(), st), "l")
t = mark("k.lookup", t)
assert torch.equal(init2, init) and torch.equal(isn.bool(), ~hit_u)
assert torch.equal(k2, keys) and torch.equal(v2, vals)
print({k: round(v, 2) for k, v in T.items()}, "total", round(sum(T.values()), 1))
