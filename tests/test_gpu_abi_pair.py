"""The same include/othello.h calls on both builds of the header: the HIP library
(device buffers, raw ctypes, no ops.py wrapper) and libothello_cpu.so (host
buffers, the oracle restatement).  Outputs must be bit-identical
(on the GPU box parity is against the fixtures and the build's
own CPU library)."""
import ctypes

import numpy as np
import pytest
import torch

import oracle
from subproc_amd import _lib
from subproc_amd.td import skeys_to_keys

pytestmark = pytest.mark.gpu

DEV = "cuda"
HOSTP = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


class Buf:
    """One logical buffer held twice: numpy (host library) and torch (device library)."""

    def __init__(self, a):
        self.h = np.ascontiguousarray(a)
        dt = {np.uint64: torch.int64, np.int64: torch.int64, np.uint8: torch.uint8, np.int8: torch.int8,
              np.int32: torch.int32, np.float64: torch.float64}[self.h.dtype.type]
        src = self.h.view(np.int64) if self.h.dtype == np.uint64 else self.h
        self.d = torch.from_numpy(src.copy()).to(dt).to(DEV)

    def device_as_host(self):
        a = self.d.cpu().numpy()
        return a.view(np.uint64) if self.h.dtype == np.uint64 else a


def both(name, *args):
    """Call `name` on both libraries; Buf arguments become host / device pointers."""
    gpu, cpu = _lib.load(), oracle.cpu_abi()
    stream = torch.cuda.current_stream().cuda_stream
    ha = [HOSTP(a.h) if isinstance(a, Buf) else a for a in args]
    da = [a.d.data_ptr() if isinstance(a, Buf) else a for a in args]
    assert getattr(cpu, name)(*ha, None) == 0, name
    assert getattr(gpu, name)(*da, stream) == 0, name
    torch.cuda.synchronize()


def both_scratch(name, *args):
    """`both` for the entry points that take caller scratch (temp, temp_bytes):
    each library's own size query, then the call with that much scratch."""
    gpu, cpu = _lib.load(), oracle.cpu_abi()
    stream = torch.cuda.current_stream().cuda_stream
    ha = [HOSTP(a.h) if isinstance(a, Buf) else a for a in args]
    da = [a.d.data_ptr() if isinstance(a, Buf) else a for a in args]
    for lib, a, st in ((cpu, ha, None), (gpu, da, stream)):
        tb = ctypes.c_size_t(0)
        assert getattr(lib, name)(*a, None, ctypes.byref(tb), st) == 0, name
        if lib is gpu:
            temp = torch.empty(max(tb.value, 1), dtype=torch.uint8, device=DEV)
            tp = temp.data_ptr()
        else:
            temp = np.zeros(max(tb.value, 1), np.uint8)
            tp = HOSTP(temp)
        assert getattr(lib, name)(*a, tp, ctypes.byref(tb), st) == 0, name
        if lib is gpu:
            torch.cuda.synchronize()


def work():
    """A rollout work word for both builds (include/othello.h: 0 at the call)."""
    return Buf(np.zeros(1, np.uint64))


def same(*bufs):
    for b in bufs:
        np.testing.assert_array_equal(b.device_as_host(), b.h)


def sort_pair(keys, vals, keys_out, vals_out, n):
    """oth_td_sort_pairs on both libraries, scratch sized by each one's query."""
    gpu, cpu = _lib.load(), oracle.cpu_abi()
    st = torch.cuda.current_stream().cuda_stream
    for lib, ptr, s in ((cpu, lambda b: HOSTP(b.h), None), (gpu, lambda b: b.d.data_ptr(), st)):
        tb = ctypes.c_size_t(0)
        assert lib.oth_td_sort_pairs(ptr(keys), ptr(vals), ptr(keys_out), ptr(vals_out), n, None,
                                     ctypes.byref(tb), s) == 0
        if lib is gpu:
            temp = torch.empty(max(tb.value, 1), dtype=torch.uint8, device=DEV)
            tp = temp.data_ptr()
        else:
            temp = np.zeros(max(tb.value, 1), np.uint8)
            tp = HOSTP(temp)
        assert lib.oth_td_sort_pairs(ptr(keys), ptr(vals), ptr(keys_out), ptr(vals_out), n, tp, ctypes.byref(tb),
                                     s) == 0
    torch.cuda.synchronize()
    same(keys_out, vals_out)


def _skeys(rng, size):
    """Random OTH_TD_SKEY values (include/othello.h): (pair, region a) << 22 |
    the regions b..h in their mixed radix, pair (discs, moves) 64 = (0, 64)
    left out (OTH_TD_KEY cannot hold it); the first and last skeys included."""
    hi = rng.integers(0, 2144 * 5, size=size, dtype=np.int64)
    hi[hi >= 64 * 5] += 5
    s = (hi << 22) | rng.integers(0, 4027725, size=size, dtype=np.int64)
    if size > 1:
        s[0], s[-1] = 0, ((2145 * 5 - 1) << 22) | (4027725 - 1)
    return s


@pytest.mark.parametrize("n,distinct", [(1, 1), (1000, 7), (300001, 5000), (2_000_003, 1 << 20)])
def test_td_sort_packed_stable(n, distinct):
    """Packed words with sort keys over the whole OTH_TD_SKEY range and many
    repeats, the payload bits (the top 28) a stream position: both builds sort
    by the skey bits alone, stably, the payload riding along."""
    rng = np.random.default_rng(n + 1)
    pool = _skeys(rng, distinct)
    k = pool[rng.integers(0, distinct, size=n)].astype(np.uint64)
    w = (np.arange(n, dtype=np.uint64) << np.uint64(_lib.TD_SKEY_BITS)) | k  # the payload: stream positions
    words, out = Buf(w), Buf(np.zeros(n, np.uint64))
    both_scratch("oth_td_sort_packed", words, out, n)
    same(out)
    np.testing.assert_array_equal(out.h, w[np.argsort(k, kind="stable")])


@pytest.mark.parametrize("n,distinct,offset", [(1, 1, 0), (4097, 7, 1), (300001, 5000, 0), (2_000_003, 1 << 20, 1),
                                               (2_000_003, 3, 0)])
def test_td_sort_unpack_pair(n, distinct, offset):
    """oth_td_sort_unpack (round 5: the sort with the unpack in its last pass)
    on both builds: the keys and values equal the stable sort of the words by
    skey bits followed by oth_td_unpack (keys: the skeys as OTH_TD_KEY values).
    Payloads as oth_td_updates_packed writes them (value_side + 64 in the top
    byte, turn_left 0..128 below); offset 1: the words start 8 bytes into a
    device buffer (not 16-B aligned)."""
    rng = np.random.default_rng(n + 7)
    pool = _skeys(rng, distinct)
    k = pool[rng.integers(0, distinct, size=n)].astype(np.uint64)
    vs = rng.integers(-64, 65, size=n).astype(np.int64)
    tl = rng.integers(0, 129, size=n).astype(np.uint64)
    w = (((vs + 64).astype(np.uint64)) << np.uint64(56)) | (tl << np.uint64(_lib.TD_PACK_TURN_SHIFT)) | k
    lam = np.array([0.9 ** j for j in range(129)], np.float64)
    words = Buf(np.concatenate([np.zeros(offset, np.uint64), w]))
    ko, vo, lamb = Buf(np.zeros(n, np.int64)), Buf(np.zeros(n, np.float64)), Buf(lam)
    gpu, cpu = _lib.load(), oracle.cpu_abi()
    st = torch.cuda.current_stream().cuda_stream
    for lib, src, ptr, s in ((cpu, HOSTP(words.h[offset:]), lambda b: HOSTP(b.h), None),
                             (gpu, words.d.data_ptr() + 8 * offset, lambda b: b.d.data_ptr(), st)):
        tb = ctypes.c_size_t(0)
        assert lib.oth_td_sort_unpack(src, ptr(lamb), ptr(ko), ptr(vo), n, None, ctypes.byref(tb), s) == 0
        temp = (torch.empty(max(tb.value, 1), dtype=torch.uint8, device=DEV) if lib is gpu
                else np.zeros(max(tb.value, 1), np.uint8))
        tp = temp.data_ptr() if lib is gpu else HOSTP(temp)
        assert lib.oth_td_sort_unpack(src, ptr(lamb), ptr(ko), ptr(vo), n, tp, ctypes.byref(tb), s) == 0
    torch.cuda.synchronize()
    same(ko, vo)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(ko.h, skeys_to_keys(k[order].astype(np.int64)))
    np.testing.assert_array_equal(vo.h, vs[order].astype(np.float64) * lam[tl[order].astype(np.int64)])


@pytest.mark.parametrize("n,distinct", [(1, 1), (1000, 7), (300001, 5000), (2_000_003, 1 << 20)])
def test_td_sort_pairs_stable(n, distinct):
    """Keys over all OTH_TD_KEY_BITS key bits with many repeats: both builds sort
    stably (values are the stream positions, so any reordering of equal keys shows)."""
    rng = np.random.default_rng(n)
    pool = rng.integers(0, 1 << _lib.TD_KEY_BITS, size=distinct, dtype=np.int64)
    pool[0] = 0
    pool[-1] = (1 << _lib.TD_KEY_BITS) - 1
    k = pool[rng.integers(0, distinct, size=n)]
    keys, vals = Buf(k), Buf(np.arange(n, dtype=np.float64))
    ko, vo = Buf(np.zeros(n, np.int64)), Buf(np.zeros(n, np.float64))
    sort_pair(keys, vals, ko, vo, n)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(ko.h, k[order])
    np.testing.assert_array_equal(vo.h, order.astype(np.float64))


@pytest.mark.parametrize("n_old,n_upd,overlap", [(0, 5, 0.0), (7, 0, 0.0), (1, 1, 1.0), (5000, 3000, 0.5),
                                                  (300_000, 1_000_000, 0.3), (2_000_000, 40_000, 0.9),
                                                  (100_000, 100_000, 1.0)])
def test_td_merge_pair(n_old, n_upd, overlap):
    """The table merge on both builds against numpy: sorted union, batch values
    where a key is in both; tiles of 2,048 merged positions, so ties and runs of
    one side cross tile and thread boundaries."""
    rng = np.random.default_rng(n_old * 7 + n_upd)
    old = np.unique(rng.integers(0, 1 << 54, size=n_old, dtype=np.int64))
    n_hit = int(overlap * min(len(old), n_upd))
    upd = np.unique(np.concatenate([rng.choice(old, size=n_hit, replace=False) if n_hit else old[:0],
                                    rng.integers(0, 1 << 54, size=n_upd - n_hit, dtype=np.int64)]))
    ov = rng.normal(size=len(old))
    uv = rng.normal(size=len(upd))
    new = ~np.isin(upd, old)
    nb = np.concatenate([[0], np.cumsum(new)]).astype(np.int64)
    n_out = len(old) + int(nb[-1])
    want = dict(zip(old.tolist(), ov.tolist()))
    want.update(zip(upd.tolist(), uv.tolist()))
    ok, ovb, uk, uvb, nbb = Buf(old), Buf(ov), Buf(upd), Buf(uv), Buf(nb)
    # the lookup that precedes the EMA: the batch keys' table values and new flags
    init, is_new = Buf(np.full(len(upd), 9.0)), Buf(np.full(len(upd), 7, np.uint8))
    both_scratch("oth_td_lookup", ok, ovb, len(old), uk, len(upd), init, is_new)
    same(init, is_new)
    np.testing.assert_array_equal(is_new.h, new.astype(np.uint8))
    olddict = dict(zip(old.tolist(), ov.tolist()))
    assert init.h.tolist() == [olddict.get(k, 0.0) for k in upd.tolist()]
    out_k, out_v = Buf(np.full(n_out, -7, np.int64)), Buf(np.zeros(n_out))
    both_scratch("oth_td_merge", ok, ovb, len(old), uk, uvb, nbb, len(upd), out_k, out_v)
    same(out_k, out_v)
    assert out_k.h.tolist() == sorted(want)
    assert out_v.h.tolist() == [want[k] for k in sorted(want)]


@pytest.mark.parametrize("n_old,n_upd,dev_count", [(40_000, 20_000, None), (40_000, 20_000, 13_001), (1, 5000, None),
                                                   (5000, 1, 1), (100_000, 70_000, 2048)])
def test_td_merge_after_lookup_pair(n_old, n_upd, dev_count):
    """oth_td_merge_after_lookup (the merge reading the merge-path splits a
    lookup left in its scratch; dev_count: the lookup was oth_td_lookup_dev
    with that device count over buffers sized for n_upd) on both builds: the
    same table as oth_td_merge, bit for bit."""
    rng = np.random.default_rng(n_old + 3 * n_upd)
    old = np.unique(rng.integers(0, 1 << 40, size=n_old, dtype=np.int64))
    upd = np.unique(np.concatenate([rng.choice(old, min(len(old), n_upd // 2), replace=False),
                                    rng.integers(0, 1 << 40, size=n_upd, dtype=np.int64)]))[:n_upd]
    m = len(upd) if dev_count is None else dev_count
    ov, uv = rng.normal(size=len(old)), rng.normal(size=len(upd))
    new = ~np.isin(upd[:m], old)
    nb = np.concatenate([[0], np.cumsum(new)]).astype(np.int64)
    n_out = len(old) + int(nb[-1])
    want = dict(zip(old.tolist(), ov.tolist()))
    want.update(zip(upd[:m].tolist(), uv[:m].tolist()))
    gpu, cpu = _lib.load(), oracle.cpu_abi()
    st = torch.cuda.current_stream().cuda_stream
    ok, ovb, uk, uvb, nbb = Buf(old), Buf(ov), Buf(upd), Buf(uv), Buf(nb)
    init, is_new = Buf(np.zeros(len(upd))), Buf(np.zeros(len(upd), np.uint8))
    cnt = Buf(np.array([m], np.int64))
    for lib, ptr, s in ((cpu, lambda b: HOSTP(b.h), None), (gpu, lambda b: b.d.data_ptr(), st)):
        tb = ctypes.c_size_t(0)
        if dev_count is None:
            args = (ptr(ok), ptr(ovb), len(old), ptr(uk), m, ptr(init), ptr(is_new))
            fn = lib.oth_td_lookup
        else:
            args = (ptr(ok), ptr(ovb), len(old), ptr(uk), len(upd), ptr(cnt), ptr(init), ptr(is_new))
            fn = lib.oth_td_lookup_dev
        assert fn(*args, None, ctypes.byref(tb), s) == 0
        temp = (torch.empty(max(tb.value, 1), dtype=torch.uint8, device=DEV) if lib is gpu
                else np.zeros(max(tb.value, 1), np.uint8))
        tp = temp.data_ptr() if lib is gpu else HOSTP(temp)
        assert fn(*args, tp, ctypes.byref(tb), s) == 0
        out_k, out_v = (np.full(n_out, -7, np.int64), np.zeros(n_out)) if lib is cpu else \
            (torch.full((n_out,), -7, dtype=torch.int64, device=DEV), torch.zeros(n_out, dtype=torch.float64, device=DEV))
        okp = HOSTP(out_k) if lib is cpu else out_k.data_ptr()
        ovp = HOSTP(out_v) if lib is cpu else out_v.data_ptr()
        assert lib.oth_td_merge_after_lookup(ptr(ok), ptr(ovb), len(old), ptr(uk), ptr(uvb), ptr(nbb), m, okp, ovp,
                                             tp, s) == 0
        if lib is gpu:
            torch.cuda.synchronize()
            out_k, out_v = out_k.cpu().numpy(), out_v.cpu().numpy()
        assert out_k.tolist() == sorted(want)
        assert out_v.tolist() == [want[k] for k in sorted(want)]


@pytest.mark.parametrize("count", [0, 1, 2047, 2048, 30_000, 50_000, 60_000])
def test_td_lookup_dev_pair(count):
    """oth_td_lookup_dev (the batch's key count read from device memory, the
    arrays and scratch sized for n_upd_max = 50,000) on both builds: the first
    `count` entries as oth_td_lookup over that many keys, the rest untouched;
    a count past n_upd_max is clamped to it."""
    rng = np.random.default_rng(count + 5)
    old = np.unique(rng.integers(0, 1 << 40, size=40_000, dtype=np.int64))
    n_max = 50_000
    upd = np.unique(np.concatenate([rng.choice(old, 20_000, replace=False),
                                    rng.integers(0, 1 << 40, size=40_000, dtype=np.int64)]))[:n_max]
    ov = rng.normal(size=len(old))
    ok, ovb, uk = Buf(old), Buf(ov), Buf(upd)
    cnt = Buf(np.array([count, 123], np.int64))
    init, is_new = Buf(np.full(n_max, 9.0)), Buf(np.full(n_max, 7, np.uint8))
    both_scratch("oth_td_lookup_dev", ok, ovb, len(old), uk, n_max, cnt, init, is_new)
    same(init, is_new)
    m = min(count, n_max)
    olddict = dict(zip(old.tolist(), ov.tolist()))
    assert init.h[:m].tolist() == [olddict.get(k, 0.0) for k in upd[:m].tolist()]
    np.testing.assert_array_equal(is_new.h[:m], (~np.isin(upd[:m], old)).astype(np.uint8))
    assert (init.h[m:] == 9.0).all() and (is_new.h[m:] == 7).all()


@pytest.mark.parametrize("shape", ["below", "above", "runs", "tiny_table"])
def test_td_merge_pair_skewed(shape):
    """Merge-path splits at the extremes (oth_td_lookup / oth_td_merge take
    their tiles' ends from a partition kernel): a batch wholly below or above
    the table, long alternating runs of each side, and a table of 3 keys
    against 700,000 batch keys."""
    rng = np.random.default_rng({"below": 1, "above": 2, "runs": 3, "tiny_table": 4}[shape])
    if shape == "below":
        old, upd = np.arange(1 << 20, (1 << 20) + 600_000) * 3, np.arange(0, 300_000) * 2
    elif shape == "above":
        old, upd = np.arange(0, 600_000) * 3, (1 << 30) + np.arange(0, 300_000) * 5
    elif shape == "runs":
        blocks = np.arange(0, 200) * 100_000
        old = np.concatenate([b + np.arange(0, 5000 + 37 * i) for i, b in enumerate(blocks[::2])])
        upd = np.concatenate([b + np.arange(0, 3000 + 11 * i) for i, b in enumerate(blocks[1::2])])
        upd = np.unique(np.concatenate([upd, rng.choice(old, 20_000, replace=False)]))
    else:
        old, upd = np.array([5, 10**9, 10**12]), np.unique(rng.integers(0, 1 << 50, 700_000))
        upd = np.unique(np.concatenate([upd, [5, 10**12]]))
    old, upd = old.astype(np.int64), upd.astype(np.int64)
    ov, uv = rng.normal(size=len(old)), rng.normal(size=len(upd))
    new = ~np.isin(upd, old)
    nb = np.concatenate([[0], np.cumsum(new)]).astype(np.int64)
    ok, ovb, uk, uvb, nbb = Buf(old), Buf(ov), Buf(upd), Buf(uv), Buf(nb)
    init, is_new = Buf(np.full(len(upd), 9.0)), Buf(np.full(len(upd), 7, np.uint8))
    both_scratch("oth_td_lookup", ok, ovb, len(old), uk, len(upd), init, is_new)
    same(init, is_new)
    np.testing.assert_array_equal(is_new.h, new.astype(np.uint8))
    n_out = len(old) + int(nb[-1])
    out_k, out_v = Buf(np.full(n_out, -7, np.int64)), Buf(np.zeros(n_out))
    both_scratch("oth_td_merge", ok, ovb, len(old), uk, uvb, nbb, len(upd), out_k, out_v)
    same(out_k, out_v)
    want = dict(zip(old.tolist(), ov.tolist()))
    want.update(zip(upd.tolist(), uv.tolist()))
    assert out_k.h.tolist() == sorted(want)


@pytest.mark.parametrize("n", [1, 1000, 3_000_001])
def test_td_fit_moments_pair(n):
    """The regression sums on both builds: the GPU's 1,024 block rows add up to
    the CPU's single row, both passes; exact for the count and the integer
    feature sums.  The float64 sums run in another order: the CPU's one
    sequential sum of 3M terms carries ~n * eps of rounding, so rtol 1e-8 and
    an absolute floor of 1e-10 of the largest sum (cross products near 0)."""
    rng = np.random.default_rng(n)
    keys = np.sort(rng.integers(0, 1 << 54, size=n, dtype=np.int64))
    vals = rng.normal(size=n)
    kb, vb = Buf(keys), Buf(vals)
    gpu, cpu = _lib.load(), oracle.cpu_abi()
    st = torch.cuda.current_stream().cuda_stream
    rows = (_lib.TD_FIT_BLOCKS, _lib.TD_FIT_COLS)
    pd, ph = torch.zeros(rows, dtype=torch.float64, device=DEV), np.zeros(rows)
    mean = None
    for width in (11, 54):
        m = None if mean is None else Buf(mean)
        assert cpu.oth_td_fit_moments(HOSTP(kb.h), HOSTP(vb.h), n, None if m is None else HOSTP(m.h), HOSTP(ph),
                                      None) == 0
        assert gpu.oth_td_fit_moments(kb.d.data_ptr(), vb.d.data_ptr(), n, None if m is None else m.d.data_ptr(),
                                      pd.data_ptr(), st) == 0
        g, c = pd[:, :width].sum(0).cpu().numpy(), ph[:, :width].sum(0)
        np.testing.assert_allclose(g, c, rtol=1e-8, atol=1e-10 * np.abs(c).max())
        if width == 11:
            np.testing.assert_array_equal(g[:10], c[:10])  # counts and integer feature sums: exact
            mean = np.append(c[1:10], c[10]) / c[0]


def positions(n, seed):
    b, t, nt, m = (Buf(np.zeros((n, 2), np.uint64)), Buf(np.zeros(n, np.uint8)), Buf(np.zeros(n, np.uint8)),
                   Buf(np.zeros(n, np.uint8)))
    both("oth_sample_midgame", seed, 0, b, t, nt, m, n)
    same(b, t, nt, m)
    return b, t, nt, m


def test_step_pair():
    n = 65536
    b, t, nt, m = positions(n, 0x5EED)
    outs = [Buf(np.zeros((n, 2), np.uint64)), Buf(np.zeros(n, np.uint8)), Buf(np.zeros(n, np.uint64)),
            Buf(np.zeros(n, np.uint64)), Buf(np.zeros(n, np.int8))]
    both("oth_step", b, t, m, *outs, nt, n)
    same(*outs, nt)
    # result + legal on the stepped boards
    res = [Buf(np.zeros(n, np.uint8)), Buf(np.zeros(n, np.uint8)), Buf(np.zeros(n, np.int8)),
           Buf(np.zeros(n, np.uint8))]
    both("oth_result", outs[0], *res, n)
    same(*res)
    leg = Buf(np.zeros(n, np.uint64))
    both("oth_legal", outs[0], outs[1], leg, n)
    same(leg)


@pytest.mark.parametrize("policy", [0, 1, 2])
def test_rollout_pair(policy):
    n = 8192
    b, t, _, _ = positions(n, 3)
    outs = [Buf(np.zeros((n, 2), np.uint64)), Buf(np.zeros(n, np.int8)), Buf(np.zeros(n, np.uint8)),
            Buf(np.zeros((n, _lib.MOVES_STRIDE), np.uint8)), Buf(np.zeros(_lib.HIST_BINS, np.int64))]
    wk = work()
    if policy == 2:
        w = (ctypes.c_int8 * 36)(*np.random.default_rng(1).integers(-127, 128, 36).tolist())
        both("oth_rollout_eval", None, None, 99, 1 << 30, 10, w, *outs, wk, n)
        both("oth_rollout_eval", b, t, 98, 5, 0, w, *outs, wk, n)  # from mid-game starts, hist accumulates
    else:
        both("oth_rollout", None, None, 99, 1 << 30, policy, 10, *outs, wk, n)
        both("oth_rollout", b, t, 98, 5, policy, 0, *outs, wk, n)
    same(*outs)
    assert int(wk.d.item()) == 0  # every launch leaves its work word at 0


@pytest.mark.parametrize("policy", [1, 2])
def test_rollout_runner_pair(policy):
    n = 4096
    b, t, _, _ = positions(n, 5)
    wa = (ctypes.c_int8 * 36)(*np.random.default_rng(11).integers(-127, 128, 36).tolist())
    wb = (ctypes.c_int8 * 36)(*np.random.default_rng(12).integers(-127, 128, 36).tolist())
    outs = [Buf(np.zeros(n, np.uint8)), Buf(np.zeros((n, 2), np.uint64)), Buf(np.zeros(n, np.int8)),
            Buf(np.zeros(n, np.uint8)), Buf(np.zeros((n, _lib.MOVES_STRIDE), np.uint8)),
            Buf(np.zeros(_lib.HIST_BINS, np.int64))]
    wk = work()
    both("oth_rollout_runner", None, None, 31, 1 << 29, policy, wa, wb, 10, 3, 1, *outs, wk, n)
    same(*outs)
    both("oth_rollout_runner", b, t, 32, 9, policy, wa, wb, 2, 12, 0, *outs, wk, n)  # mid-game starts, no swap
    same(*outs)
    assert int(wk.d.item()) == 0


def test_books_features_eval_pair():
    n = 512
    outs = [None, None, Buf(np.zeros(n, np.uint8)), Buf(np.full((n, _lib.MOVES_STRIDE), 255, np.uint8)), None]
    both("oth_rollout", None, None, 5, 0, 0, 0, None, None, outs[2], outs[3], None, work(), n)
    same(outs[2], outs[3])
    pos = Buf(np.full((n, _lib.POS_STRIDE, 2), 0x5A5A5A5A5A5A5A5A, np.uint64))
    pt, pe = Buf(np.full((n, _lib.POS_STRIDE), 0xAB, np.uint8)), Buf(np.full((n, _lib.POS_STRIDE), 0xCD, np.uint8))
    both("oth_replay", None, None, outs[3], outs[2], pos, pt, pe, n)
    # every row is written by both: board, turn and end rows past plies as 0
    same(pos, pt, pe)
    rows = outs[2].h.astype(np.int64) + 1
    off = Buf(np.cumsum(rows) - rows)
    pk = [Buf(np.zeros((int(rows.sum()), 2), np.uint64)), Buf(np.zeros(int(rows.sum()), np.uint8)),
          Buf(np.zeros(int(rows.sum()), np.uint8))]
    both("oth_replay_rows", None, None, outs[3], outs[2], off, *pk, n)
    same(*pk)
    past = np.arange(_lib.POS_STRIDE)[None, :] > outs[2].h[:, None]
    assert (pos.h[past] == 0).all() and (pt.h[past] == 0).all() and (pe.h[past] == 0).all()
    k = n * _lib.POS_STRIDE
    flat_b = Buf(pos.h.reshape(k, 2))
    flat_t = Buf(pt.h.reshape(k))
    txt = Buf(np.zeros(k * _lib.BOOK_LINE, np.uint8))
    both("oth_book_text", flat_b, flat_t, k, txt)
    same(txt)
    side = Buf(np.random.default_rng(2).integers(0, 4, k).astype(np.uint8))
    feats = Buf(np.zeros((k, _lib.N_FEATURES), np.uint8))
    both("oth_features", flat_b, side, feats, k)
    ev = Buf(np.zeros(k, np.int32))
    w = (ctypes.c_int8 * 36)(*np.random.default_rng(3).integers(-128, 128, 36).tolist())
    both("oth_eval", flat_b, side, w, ev, k)
    same(feats, ev)


def test_td_pair():
    n = 256
    plies = Buf(np.zeros(n, np.uint8))
    moves = Buf(np.full((n, _lib.MOVES_STRIDE), 255, np.uint8))
    both("oth_rollout", None, None, 21, 0, 1, 4, None, None, plies, moves, None, work(), n)
    same(plies, moves)
    pos = Buf(np.zeros((n, _lib.POS_STRIDE, 2), np.uint64))
    both("oth_replay", None, None, moves, plies, pos, None, None, n)
    same(pos)
    cnt = 2 * (plies.h.astype(np.int64) + 1)
    base = Buf(np.cumsum(cnt) - cnt)
    lam = Buf(np.array([0.9 ** k for k in range(_lib.POS_STRIDE)], np.float64))
    total = int(cnt.sum())
    keys, vals = Buf(np.zeros(total, np.int64)), Buf(np.zeros(total, np.float64))
    both("oth_td_updates", pos, plies, base, lam, keys, vals, n)
    same(keys, vals)
    # the packed-rows layout: oth_replay_rows + oth_td_updates_rows give the same stream
    rows = plies.h.astype(np.int64) + 1
    off = Buf(np.cumsum(rows) - rows)
    prow = Buf(np.zeros((int(rows.sum()), 2), np.uint64))
    both("oth_replay_rows", None, None, moves, plies, off, prow, None, None, n)
    same(prow)
    keys2, vals2 = Buf(np.zeros(total, np.int64)), Buf(np.zeros(total, np.float64))
    both("oth_td_updates_rows", prow, off, plies, base, lam, keys2, vals2, n)
    same(keys2, vals2)
    np.testing.assert_array_equal(keys2.h, keys.h)
    np.testing.assert_array_equal(vals2.h.view(np.int64), vals.h.view(np.int64))
    order = np.argsort(keys.h, kind="stable")
    uk, starts = np.unique(keys.h[order], return_index=True)
    sv = Buf(vals.h[order])
    # the grouping sort: both builds give numpy's stable order, bit for bit
    sk2, sv2 = Buf(np.zeros(total, np.int64)), Buf(np.zeros(total, np.float64))
    sort_pair(keys, vals, sk2, sv2, total)
    np.testing.assert_array_equal(sk2.h, keys.h[order])
    np.testing.assert_array_equal(sv2.h.view(np.int64), sv.h.view(np.int64))
    # the packed path (StateMap.update): the same stream as words, sorted by
    # their key bits with the payload riding along, unpacked -> the same
    # sorted keys and values, bit for bit, on both builds and both layouts
    for po, layout in ((None, pos), (off, prow)):
        words = Buf(np.zeros(total, np.uint64))
        both("oth_td_updates_packed", layout, po, plies, base, words, n)
        same(words)
        np.testing.assert_array_equal(skeys_to_keys((words.h & np.uint64((1 << _lib.TD_SKEY_BITS) - 1)).astype(np.int64)),
                                      keys.h)
        sw = Buf(np.zeros(total, np.uint64))
        both_scratch("oth_td_sort_packed", words, sw, total)
        same(sw)
        uk2, uv2 = Buf(np.zeros(total, np.int64)), Buf(np.zeros(total, np.float64))
        both("oth_td_unpack", sw, lam, uk2, uv2, total)
        same(uk2, uv2)
        np.testing.assert_array_equal(uk2.h, keys.h[order])
        np.testing.assert_array_equal(uv2.h.view(np.int64), sv.h.view(np.int64))
    seg = Buf(np.append(starts, total).astype(np.int64))
    init = Buf(np.random.default_rng(4).choice([0.0, 0.5, -1.25], len(uk)))
    out = Buf(np.zeros(len(uk), np.float64))
    both("oth_td_ema", sv, seg, init, 0.03, 1 - 0.03, out, len(uk))
    same(out)
    lens = np.diff(seg.h)
    li = Buf(np.flatnonzero(lens >= 48).astype(np.int64))
    assert 0 < len(li.h) < len(uk)
    out2 = Buf(np.zeros(len(uk), np.float64))
    both_scratch("oth_td_ema_split", sv, seg, init, 0.03, 1 - 0.03, out2, len(uk), 48, li, len(li.h), total)
    same(out2)
    np.testing.assert_array_equal(out2.h, out.h)


def test_td_updates_ragged_long_pair():
    """The update stream for a game count that is no multiple of the kernel's
    games per wave (OTH_TD_UPD_GAMES) and for games of 0 to 128 plies (positions
    64 and on take the lanes' second round): synthetic disjoint boards, every
    layout and output form, both builds bit for bit."""
    rng = np.random.default_rng(11)
    pl = np.array([0, 1, 5, 63, 64, 65, 127, 128, 60, 2, 100], np.uint8)
    n = len(pl)
    b = rng.integers(0, 2 ** 63, (n, _lib.POS_STRIDE), dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, (n, _lib.POS_STRIDE), dtype=np.uint64)
    w = rng.integers(0, 2 ** 63, (n, _lib.POS_STRIDE), dtype=np.uint64) & ~b
    pos = Buf(np.stack([b, w], axis=-1))
    rows = pl.astype(np.int64) + 1
    off = Buf(np.cumsum(rows) - rows)
    prow = Buf(np.concatenate([pos.h[g, :rows[g]] for g in range(n)]))
    plies = Buf(pl)
    cnt = 2 * rows
    base = Buf(np.cumsum(cnt) - cnt)
    total = int(cnt.sum())
    lam = Buf(np.array([0.9 ** k for k in range(_lib.POS_STRIDE)], np.float64))
    keys, vals = Buf(np.zeros(total, np.int64)), Buf(np.zeros(total, np.float64))
    both("oth_td_updates", pos, plies, base, lam, keys, vals, n)
    same(keys, vals)
    keys2, vals2 = Buf(np.zeros(total, np.int64)), Buf(np.zeros(total, np.float64))
    both("oth_td_updates_rows", prow, off, plies, base, lam, keys2, vals2, n)
    same(keys2, vals2)
    np.testing.assert_array_equal(keys2.h, keys.h)
    for po, layout in ((None, pos), (off, prow)):
        words = Buf(np.zeros(total, np.uint64))
        both("oth_td_updates_packed", layout, po, plies, base, words, n)
        same(words)
        np.testing.assert_array_equal(skeys_to_keys((words.h & np.uint64((1 << _lib.TD_SKEY_BITS) - 1)).astype(np.int64)),
                                      keys.h)


@pytest.mark.parametrize("long_min", [48, 1, 2, 64, 65, 66, 1000])
def test_td_segments_pair(long_min):
    """oth_td_segments: the runs of a key-sorted stream (short, long, a
    single-key stream's one run, runs crossing the GPU's 64-key rounds and
    1,024-key waves) -- offsets and keys equal on both builds and to numpy's,
    the long segments the same set.  long_min up to 65 takes the GPU's
    register path (the key long_min - 1 places on by __shfl, round 5), beyond
    it the load from memory."""
    rng = np.random.default_rng(12)
    for lens in (rng.integers(1, 5, 3000), np.array([70000]), rng.choice([1, 2, 47, 48, 49, 63, 64, 65, 66, 1023, 1024,
                                                                           1025, 5000], 400)):
        keys = np.repeat(np.cumsum(rng.integers(1, 1000, len(lens))).astype(np.int64), lens)
        n = len(keys)
        k = Buf(keys)
        off, uk, li, cnt = (Buf(np.zeros(n + 1, np.int64)), Buf(np.zeros(n, np.int64)), Buf(np.zeros(n, np.int64)),
                            Buf(np.zeros(2, np.int64)))
        both_scratch("oth_td_segments", k, n, long_min, off, uk, li, cnt)
        same(cnt)
        m, nl = (int(x) for x in cnt.h)
        starts = np.flatnonzero(np.r_[True, keys[1:] != keys[:-1]])
        assert m == len(starts)
        np.testing.assert_array_equal(off.h[:m + 1], np.r_[starts, n])
        np.testing.assert_array_equal(uk.h[:m], keys[starts])
        np.testing.assert_array_equal(off.d.cpu().numpy()[:m + 1], off.h[:m + 1])
        np.testing.assert_array_equal(uk.d.cpu().numpy()[:m], uk.h[:m])
        want = np.flatnonzero(np.diff(np.r_[starts, n]) >= long_min)
        assert nl == len(want)
        np.testing.assert_array_equal(li.h[:nl], want)
        np.testing.assert_array_equal(np.sort(li.d.cpu().numpy()[:nl]), want)


def word_errors(reset=False):
    """oth_td_word_errors on both builds: (device count, host count)."""
    gpu, cpu = _lib.load(), oracle.cpu_abi()
    g, c = ctypes.c_uint64(0), ctypes.c_uint64(0)
    assert gpu.oth_td_word_errors(ctypes.byref(g), int(reset), torch.cuda.current_stream().cuda_stream) == 0
    assert cpu.oth_td_word_errors(ctypes.byref(c), int(reset), None) == 0
    return int(g.value), int(c.value)


def test_td_unpack_clamps_turn_left_pair():
    """Words whose turn_left exceeds 128 (not from oth_td_updates_packed):
    both builds read lam_pow[128], in oth_td_unpack, oth_td_segments_words and
    oth_td_sort_unpack, never past the table, and count every such word read
    (oth_td_word_errors) instead of hiding it."""
    word_errors(reset=True)
    lam = Buf(np.array([0.9 ** j for j in range(129)], np.float64))
    tl = np.array([0, 128, 129, 0xFFFFF] * 16, np.uint64)
    w = Buf((np.uint64(64 - 5) << np.uint64(56)) | (tl << np.uint64(_lib.TD_PACK_TURN_SHIFT)))
    n = len(tl)
    bad = int((tl > 128).sum())
    keys, vals = Buf(np.zeros(n, np.int64)), Buf(np.zeros(n, np.float64))
    both("oth_td_unpack", w, lam, keys, vals, n)
    same(keys, vals)
    np.testing.assert_array_equal(vals.h, -5.0 * lam.h[np.minimum(tl, 128).astype(np.int64)])
    assert word_errors() == (bad, bad)
    off, uk, li, cnt, val = (Buf(np.zeros(n + 1, np.int64)), Buf(np.zeros(n, np.int64)), Buf(np.zeros(n, np.int64)),
                             Buf(np.zeros(2, np.int64)), Buf(np.zeros(n, np.float64)))
    both_scratch("oth_td_segments_words", w, lam, n, 48, off, uk, li, cnt, val)
    same(cnt, val)
    np.testing.assert_array_equal(val.h, vals.h)
    assert word_errors() == (2 * bad, 2 * bad)
    ko, vo = Buf(np.zeros(n, np.int64)), Buf(np.zeros(n, np.float64))
    both_scratch("oth_td_sort_unpack", w, lam, ko, vo, n)
    same(ko, vo)
    assert word_errors(reset=True) == (3 * bad, 3 * bad)
    assert word_errors() == (0, 0)


def test_td_word_errors_zero_on_the_learner_path():
    """A StateMap update over real GPU books (oth_td_updates_packed words through
    the sort, the segments and the EMA) reads no out-of-range word; a corrupted
    copy of its words is reported."""
    from subproc_amd import ops
    from subproc_amd.td import StateMap, lam_pow_table, word_errors as td_word_errors

    td_word_errors(reset=True)
    r = ops.rollout(4096, 0x5EED, 0, "random", record_moves=True, device=DEV)
    sm = StateMap(DEV)
    sm.update_rows(ops.replay_rows(r.moves, r.plies), r.plies)
    assert len(sm) > 0 and td_word_errors() == 0
    w = torch.randint(0, 1 << 36, (1000,), dtype=torch.int64, device=DEV)
    w[::10] |= 300 << _lib.TD_PACK_TURN_SHIFT  # 100 words with turn_left 300
    lam = torch.tensor(lam_pow_table(), dtype=torch.float64, device=DEV)
    k, v = torch.empty_like(w), torch.empty(1000, dtype=torch.float64, device=DEV)
    _lib.check(_lib.load().oth_td_unpack(w.data_ptr(), lam.data_ptr(), k.data_ptr(), v.data_ptr(), 1000,
                                         torch.cuda.current_stream().cuda_stream), "oth_td_unpack")
    assert td_word_errors() == 100 and td_word_errors() == 0


def test_td_segments_words_pair():
    """oth_td_segments_words (round 5): the same runs read from skey-sorted
    packed words (payloads in the top 28 bits, which must not split a run),
    the keys handed back as OTH_TD_KEY values, and every word's value as
    oth_td_unpack gives it, on both builds."""
    rng = np.random.default_rng(13)
    lam = np.array([0.9 ** j for j in range(129)], np.float64)
    for lens in (rng.integers(1, 5, 3000), np.array([70000]), rng.choice([1, 2, 47, 48, 49, 1023, 1024, 1025, 5000],
                                                                          400)):
        keys = np.repeat(np.sort(_skeys(rng, len(lens))).astype(np.uint64), lens)  # sorted skeys
        n = len(keys)
        vs = rng.integers(-64, 65, n).astype(np.int64)
        tl = rng.integers(0, 129, n).astype(np.uint64)
        w = ((vs + 64).astype(np.uint64) << np.uint64(56)) | (tl << np.uint64(_lib.TD_PACK_TURN_SHIFT)) | keys
        words, lamb = Buf(w), Buf(lam)
        off, uk, li, cnt, val = (Buf(np.zeros(n + 1, np.int64)), Buf(np.zeros(n, np.int64)),
                                 Buf(np.zeros(n, np.int64)), Buf(np.zeros(2, np.int64)), Buf(np.zeros(n, np.float64)))
        both_scratch("oth_td_segments_words", words, lamb, n, 48, off, uk, li, cnt, val)
        same(cnt, val)
        m, nl = (int(x) for x in cnt.h)
        starts = np.flatnonzero(np.r_[True, keys[1:] != keys[:-1]])
        assert m == len(starts)
        np.testing.assert_array_equal(off.h[:m + 1], np.r_[starts, n])
        np.testing.assert_array_equal(off.d.cpu().numpy()[:m + 1], off.h[:m + 1])
        np.testing.assert_array_equal(uk.d.cpu().numpy()[:m], skeys_to_keys(keys[starts].astype(np.int64)))
        np.testing.assert_array_equal(uk.h[:m], uk.d.cpu().numpy()[:m])
        np.testing.assert_array_equal(val.h, vs.astype(np.float64) * lam[tl.astype(np.int64)])
        want = np.flatnonzero(np.diff(np.r_[starts, n]) >= 48)
        assert nl == len(want)
        np.testing.assert_array_equal(np.sort(li.d.cpu().numpy()[:nl]), want)


def test_td_new_before_pair():
    """oth_td_new_before: the running count of a byte flag array (empty, short,
    across the GPU's 64-flag rounds and 1,024-flag waves), equal on both builds
    and to numpy's."""
    rng = np.random.default_rng(13)
    for n in (0, 1, 63, 64, 65, 1023, 1024, 1025, 200_003):
        f = (rng.random(n) < 0.4).astype(np.uint8) * rng.integers(1, 255, n).astype(np.uint8)
        fl = Buf(f if n else np.zeros(1, np.uint8))
        nb = Buf(np.zeros(n + 1, np.int64))
        both_scratch("oth_td_new_before", fl, n, nb)
        same(nb)
        np.testing.assert_array_equal(nb.h, np.r_[0, np.cumsum(f[:n] != 0)])


def test_empty_null_and_invalid_arguments():
    """n = 0 is a no-op for every entry point; optional outputs may be NULL;
    bad arguments return OTH_EINVAL before anything is launched (both builds)."""
    gpu, cpu = _lib.load(), oracle.cpu_abi()
    st = torch.cuda.current_stream().cuda_stream
    w = (ctypes.c_int8 * 36)()
    wk = work()
    for lib, s, W in ((gpu, st, wk.d.data_ptr()), (cpu, None, HOSTP(wk.h))):
        assert lib.oth_reset(None, None, None, 0, s) == 0
        assert lib.oth_legal(None, None, None, 0, s) == 0
        assert lib.oth_step(None, None, None, None, None, None, None, None, None, 0, s) == 0
        assert lib.oth_result(None, None, None, None, None, 0, s) == 0
        assert lib.oth_rollout(None, None, 1, 0, 0, 0, None, None, None, None, None, W, 0, s) == 0
        assert lib.oth_rollout_eval(None, None, 1, 0, 0, w, None, None, None, None, None, W, 0, s) == 0
        assert lib.oth_rollout_match(None, None, 1, 0, 0, w, w, None, None, None, None, None, W, 0, s) == 0
        assert lib.oth_hands(None, None, None, None, None, None, None, 0, s) == 0
        assert lib.oth_replay(None, None, None, None, None, None, None, 0, s) == 0
        assert lib.oth_replay_rows(None, None, None, None, None, None, None, None, 0, s) == 0
        assert lib.oth_replay_rows(None, None, None, None, None, None, None, None, 3, s) == _lib.OTH_EINVAL
        assert lib.oth_td_updates_rows(None, None, None, None, None, None, None, 0, s) == 0
        assert lib.oth_rollout_runner(None, None, 1, 0, 1, None, None, 0, 0, 0, None, None, None, None, None, None,
                                      W, 0, s) == 0
        assert lib.oth_rollout_runner(None, None, 1, 0, 0, w, w, 0, 0, 0, None, None, None, None, None, None,
                                      W, 5, s) == _lib.OTH_EINVAL  # random is not a runner policy
        assert lib.oth_book_text(None, None, 0, None, s) == 0
        assert lib.oth_features(None, None, None, 0, s) == 0
        assert lib.oth_eval(None, None, w, None, 0, s) == 0
        assert lib.oth_td_updates(None, None, None, None, None, None, 0, s) == 0
        assert lib.oth_td_ema(None, None, None, 0.03, 0.97, None, 0, s) == 0
        tb0 = ctypes.c_size_t(0)
        assert lib.oth_td_ema_split(None, None, None, 0.03, 0.97, None, 0, 1, None, 0, 0, None, ctypes.byref(tb0),
                                    s) == 0  # size query
        assert lib.oth_td_ema_split(None, None, None, 0.03, 0.97, None, 0, 1, None, 0, 0, ctypes.c_void_p(8),
                                    ctypes.byref(tb0), s) == 0
        assert lib.oth_sample_midgame(1, 0, None, None, None, None, 0, s) == 0
        E = _lib.OTH_EINVAL
        assert lib.oth_step(None, None, None, None, None, None, None, None, None, 5, s) == E
        assert lib.oth_rollout(None, None, 1, 0, 3, 0, None, None, None, None, None, W, 5, s) == E  # bad policy
        assert lib.oth_rollout(None, None, 1, 0, 0, 0, None, None, None, None, None, W, -1, s) == E
        assert lib.oth_rollout(None, None, 1, 0, 0, 0, None, None, None, None, None, None, 5, s) == E  # no work word
        assert lib.oth_rollout_eval(None, None, 1, 0, 0, None, None, None, None, None, None, W, 5, s) == E
        assert lib.oth_rollout_eval(None, None, 1, 0, 0, w, None, None, None, None, None, None, 5, s) == E
        assert lib.oth_rollout_match(None, None, 1, 0, 0, w, None, None, None, None, None, None, W, 5, s) == E
        assert lib.oth_hands(None, None, None, None, None, None, None, 3, s) == E
        assert lib.oth_eval(None, None, None, None, 0, s) == E
        assert lib.oth_td_ema(None, None, None, 0.03, 0.97, None, 3, s) == E
        tb0 = ctypes.c_size_t(0)
        assert lib.oth_td_ema_split(None, None, None, 0.03, 0.97, None, 0, 0, None, 0, 0, None, ctypes.byref(tb0),
                                    s) == E  # long_min < 1
        assert lib.oth_td_ema_split(None, None, None, 0.03, 0.97, None, 0, 1, None, 0, 0, None, None, s) == E  # no size
        tb = ctypes.c_size_t(0)
        assert lib.oth_td_sort_pairs(None, None, None, None, 0, None, ctypes.byref(tb), s) == 0  # size query
        assert lib.oth_td_sort_pairs(None, None, None, None, 0, ctypes.c_void_p(8), ctypes.byref(tb), s) == 0
        assert lib.oth_td_sort_pairs(None, None, None, None, -1, None, ctypes.byref(tb), s) == E
        assert lib.oth_td_sort_pairs(None, None, None, None, 5, None, None, s) == E  # no size
        assert lib.oth_td_sort_pairs(None, None, None, None, 5, ctypes.c_void_p(8), ctypes.byref(tb), s) == E
        tb, one = ctypes.c_size_t(0), ctypes.c_void_p(8)
        assert lib.oth_td_merge(None, None, 0, None, None, None, 0, None, None, one, ctypes.byref(tb), s) == 0
        assert lib.oth_td_merge(None, None, 0, None, None, None, 0, None, None, one, None, s) == E  # no size
        assert lib.oth_td_lookup(None, None, 5, None, 0, None, None, one, ctypes.byref(tb), s) == E  # table w/o pointers
        assert lib.oth_td_lookup(None, None, 0, None, 0, None, None, one, ctypes.byref(tb), s) == 0
        assert lib.oth_td_lookup(None, None, 0, None, 3, None, None, one, ctypes.byref(tb), s) == E
        # the device-count form: no count pointer with keys to look up
        assert lib.oth_td_lookup_dev(None, None, 0, one, 3, None, one, one, one, ctypes.byref(tb), s) == E
        assert lib.oth_td_lookup_dev(None, None, 0, None, -1, one, None, None, one, ctypes.byref(tb), s) == E
        assert lib.oth_td_lookup_dev(None, None, 10_000, None, 7_000, None, None, None, None, ctypes.byref(tb), s) == 0
        # size queries read nothing but the counts
        assert lib.oth_td_lookup(None, None, 10_000, None, 7_000, None, None, None, ctypes.byref(tb), s) == 0
        assert tb.value >= 8 or lib is not _lib.load()
        assert lib.oth_td_merge(None, None, 10_000, None, None, None, 7_000, None, None, None, ctypes.byref(tb), s) == 0
        assert lib.oth_td_fit_moments(None, None, 3, None, ctypes.c_void_p(8), s) == E
        assert lib.oth_td_fit_moments(None, None, 0, None, None, s) == E  # no partials
        assert lib.oth_td_merge(None, None, -1, None, None, None, 0, None, None, one, ctypes.byref(tb), s) == E
        assert lib.oth_td_merge(None, None, 3, None, None, None, 0, None, None, one, ctypes.byref(tb), s) == E
        assert lib.oth_td_merge(None, None, 0, None, None, None, 3, None, None, one, ctypes.byref(tb), s) == E
    # a batch with no keys: the table is copied, new_before is not needed (NULL)
    old = Buf(np.array([3, 8, 40], np.int64))
    ov = Buf(np.array([0.5, -2.0, 7.25]))
    ok, ovo = Buf(np.zeros(3, np.int64)), Buf(np.zeros(3))
    both_scratch("oth_td_merge", old, ov, 3, None, None, None, 0, ok, ovo)
    same(ok, ovo)
    assert ok.h.tolist() == [3, 8, 40] and ovo.h.tolist() == [0.5, -2.0, 7.25]
    # every rollout output may be NULL: only the histogram is produced
    n = 4096
    hist = Buf(np.zeros(_lib.HIST_BINS, np.int64))
    both("oth_rollout", None, None, 12, 0, 0, 10, None, None, None, None, hist, work(), n)
    same(hist)
    assert int(hist.h[:129].sum()) == n
