"""TD state map (progress_position_moves_learn.py:37-62):
host side — key packing, the oracle restatement and the CPU build of the
header's oth_td_* against the fixture made with the reference's hash_from_book."""
import ctypes

import numpy as np
import pytest

import oracle
from golden_io import load_npz
from subproc_amd import _lib, td

P = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


def fixture():
    z = load_npz("td_state.npz")
    return {tuple(int(x) for x in h.split(":")): float(v) for h, v in zip(z["hash"], z["value"])}


def fixture_games():
    z = load_npz("rollout_random.npz")
    pos = oracle.replay(z["moves"], z["plies"])
    return pos["boards"], z["plies"]


def test_key_packing():
    # every field at its largest value: discs 64, moves 63, the region sizes
    for c in [(4, 4, 0, 0, 0, 0, 0, 0, 0, 2), (64, 0, 4, 8, 4, 8, 8, 16, 4, 12), (64, 63, 0, 0, 0, 0, 0, 0, 0, 0),
              (64, 63, 4, 8, 4, 8, 8, 16, 4, 12)]:
        k = td.counts_to_key(c)
        assert td.key_to_counts(k) == c and k < (1 << _lib.TD_KEY_BITS)
        assert td.hash_string(k) == ":".join(map(str, c))
    # integer order == tuple order
    cs = [(5, 3, 1, 0, 0, 0, 0, 0, 0, 0), (5, 3, 0, 8, 4, 8, 8, 16, 4, 12), (4, 40, 4, 8, 4, 8, 8, 16, 4, 12),
          (5, 2, 4, 8, 4, 8, 8, 16, 4, 12), (5, 3, 0, 8, 4, 8, 8, 16, 4, 11)]
    assert sorted(cs) == sorted(cs, key=td.counts_to_key)
    for bad in [(128, 0, 0, 0, 0, 0, 0, 0, 0, 0), (4, 64, 0, 0, 0, 0, 0, 0, 0, 0), (4, 4, 8, 0, 0, 0, 0, 0, 0, 0)]:
        with pytest.raises(ValueError):
            td.counts_to_key(bad)


def test_lam_pow_is_cpython_pow():
    t = td.lam_pow_table()
    assert t[0] == 1.0 and t[1] == 0.9 and t[61] == 0.9 ** 61 and len(t) == _lib.POS_STRIDE


def test_oracle_state_map_matches_reference_fixture():
    boards, plies = fixture_games()
    got = oracle.td_state_map(boards, plies)
    assert got == fixture()  # float equality: bit-exact


def test_cpu_abi_td_matches_fixture_and_batches_compose():
    boards, plies = fixture_games()
    lib = oracle.cpu_abi()
    lam = np.array(td.lam_pow_table(), np.float64)

    def run(b, pl, state):
        n = len(pl)
        cnt = 2 * (pl.astype(np.int64) + 1)
        base = np.ascontiguousarray(np.cumsum(cnt) - cnt)
        keys, vals = np.empty(int(cnt.sum()), np.int64), np.empty(int(cnt.sum()), np.float64)
        assert lib.oth_td_updates(P(np.ascontiguousarray(b)), P(np.ascontiguousarray(pl)), P(base), P(lam), P(keys),
                                  P(vals), n, None) == 0
        # the grouping sort through the ABI (size query, then the sort), as StateMap.update
        sk, sv = np.empty_like(keys), np.empty_like(vals)
        tb = ctypes.c_size_t(0)
        assert lib.oth_td_sort_pairs(P(keys), P(vals), P(sk), P(sv), len(keys), None, ctypes.byref(tb), None) == 0
        temp = np.empty(tb.value, np.uint8)
        assert lib.oth_td_sort_pairs(P(keys), P(vals), P(sk), P(sv), len(keys), P(temp), ctypes.byref(tb), None) == 0
        order = np.argsort(keys, kind="stable")
        np.testing.assert_array_equal(sk, keys[order])
        np.testing.assert_array_equal(sv, vals[order])
        uk, starts, counts = np.unique(sk, return_index=True, return_counts=True)
        seg = np.ascontiguousarray(np.append(starts, len(sk)).astype(np.int64))
        init = np.ascontiguousarray([state.get(int(k), 0.0) for k in uk], np.float64)
        out = np.empty(len(uk), np.float64)
        assert lib.oth_td_ema(P(sv), P(seg), P(init), 0.03, 1 - 0.03, P(out), len(uk), None) == 0
        state.update({int(k): float(v) for k, v in zip(uk, out)})
        return state

    want = {td.counts_to_key(k): v for k, v in fixture().items()}
    assert run(boards, plies, {}) == want
    s = run(boards[:100], plies[:100], {})
    assert run(boards[100:], plies[100:], s) == want


def test_fit_matches_sklearn_on_fixture_states():
    """StateMap.fit's algorithm through the CPU build of oth_td_fit_moments
    (shard = contiguous range of the key-sorted table; pass 1 means, pass 2
    centred cross products; minimum-norm solve) == sklearn
    LinearRegression(fit_intercept=True) per shard (fit_parameter,
    progress_position_moves_learn.py:160-184) on the same states; float64,
    tolerance rtol 1e-6 / atol 1e-9 on the coefficients."""
    from sklearn import linear_model

    f = fixture()
    lib = oracle.cpu_abi()
    keys = np.array(sorted(td.counts_to_key(k) for k in f), np.int64)
    vals = np.array([f[td.key_to_counts(k)] for k in keys.tolist()], np.float64)
    part = np.zeros((_lib.TD_FIT_BLOCKS, _lib.TD_FIT_COLS))
    coef, icpt, n = np.zeros((4, 9)), np.zeros(4), np.zeros(4, np.int64)
    for k, (lo, hi) in enumerate(td.SHARDS):
        s, e = np.searchsorted(keys, [lo << td._SHIFTS[0], (hi + 1) << td._SHIFTS[0]])
        n[k] = e - s
        if e == s:
            continue
        kp, vp = np.ascontiguousarray(keys[s:e]), np.ascontiguousarray(vals[s:e])
        assert lib.oth_td_fit_moments(P(kp), P(vp), e - s, None, P(part), None) == 0
        m1 = part[:, :11].sum(0)
        assert m1[0] == e - s
        mean = np.ascontiguousarray(np.append(m1[1:10], m1[10]) / m1[0])
        assert lib.oth_td_fit_moments(P(kp), P(vp), e - s, P(mean), P(part), None) == 0
        m2 = part[:, :54].sum(0)
        A = np.zeros((9, 9))
        A[np.triu_indices(9)] = m2[:45]
        A = A + np.triu(A, 1).T
        coef[k] = np.linalg.lstsq(A, m2[45:], rcond=None)[0]
        icpt[k] = mean[9] - mean[:9] @ coef[k]
    assert n.sum() == len(keys)
    for k, (lo, hi) in enumerate(td.SHARDS):
        rows = [(c, v) for c, v in f.items() if lo <= c[0] <= hi]
        assert len(rows) == n[k]
        if len(rows) < 2:
            continue
        X = np.array([c[1:] for c, _ in rows], np.float64)
        y = np.array([v for _, v in rows])
        lr = linear_model.LinearRegression(fit_intercept=True).fit(X, y)
        np.testing.assert_allclose(coef[k], lr.coef_, rtol=1e-6, atol=1e-9)
        np.testing.assert_allclose(icpt[k], lr.intercept_, rtol=1e-6, atol=1e-9)


def test_cpu_abi_td_merge():
    """The CPU build's table merge: sorted union, batch values where a key is in
    both, and OTH_EINVAL when new_before does not add up."""
    lib = oracle.cpu_abi()
    rng = np.random.default_rng(3)
    old = np.unique(rng.integers(0, 1 << 54, size=5000, dtype=np.int64))
    upd = np.unique(np.concatenate([rng.choice(old, 1000, replace=False), rng.integers(0, 1 << 54, 2000)]))
    ov, uv = rng.normal(size=len(old)), rng.normal(size=len(upd))
    nb = np.concatenate([[0], np.cumsum(~np.isin(upd, old))]).astype(np.int64)
    n_out = len(old) + int(nb[-1])
    ok, vals = np.empty(n_out, np.int64), np.empty(n_out)
    tb = ctypes.c_size_t(7)
    assert lib.oth_td_merge(P(old), P(ov), len(old), P(upd), P(uv), P(nb), len(upd), P(ok), P(vals), None,
                            ctypes.byref(tb), None) == 0 and tb.value == 0  # the host build needs no scratch
    tmp = np.zeros(1, np.uint8)
    assert lib.oth_td_merge(P(old), P(ov), len(old), P(upd), P(uv), P(nb), len(upd), P(ok), P(vals), P(tmp),
                            ctypes.byref(tb), None) == 0
    want = dict(zip(old.tolist(), ov.tolist()))
    want.update(zip(upd.tolist(), uv.tolist()))
    assert ok.tolist() == sorted(want) and vals.tolist() == [want[k] for k in sorted(want)]
    nb[-1] -= 1  # one new key too few: the output would overflow
    assert lib.oth_td_merge(P(old), P(ov), len(old), P(upd), P(uv), P(nb), len(upd), P(ok), P(vals), P(tmp),
                            ctypes.byref(tb), None) == _lib.OTH_EINVAL


def test_cpu_abi_td_lookup():
    lib = oracle.cpu_abi()
    old = np.array([2, 5, 9, 11], np.int64)
    ov = np.array([0.5, -1.0, 2.0, 3.5])
    upd = np.array([1, 5, 10, 11, 12], np.int64)
    init, is_new = np.full(5, 9.0), np.full(5, 7, np.uint8)
    tb, tmp = ctypes.c_size_t(0), np.zeros(1, np.uint8)
    assert lib.oth_td_lookup(P(old), P(ov), 4, P(upd), 5, P(init), P(is_new), P(tmp), ctypes.byref(tb), None) == 0
    assert init.tolist() == [0.0, -1.0, 0.0, 3.5, 0.0] and is_new.tolist() == [1, 0, 1, 0, 1]


def test_skey_order_and_round_trip():
    """include/othello.h OTH_TD_SKEY (the packed words' 36-bit sort key): a
    bijection on counts() tuples with moves <= 64 - discs that orders them as
    OTH_TD_KEY does, decoded alike by the scalar and the vectorised helper;
    every skey fits 36 bits."""
    rng = np.random.default_rng(5)
    cs = [(0,) * 10, (64, 0, 4, 8, 4, 8, 8, 16, 4, 12), (0, 63, 4, 8, 4, 8, 8, 16, 4, 12), (1, 63) + (0,) * 8]
    for _ in range(5000):
        d = int(rng.integers(0, 65))
        cs.append((d, int(rng.integers(0, min(64, 65 - d)))) + tuple(int(rng.integers(0, b)) for b in (5, 9, 5, 9, 9, 17, 5, 13)))
    keys = np.array([td.counts_to_key(c) for c in cs])
    skeys = np.array([td.counts_to_skey(c) for c in cs])
    assert all(td.skey_to_counts(s) == tuple(c) for s, c in zip(skeys, cs))
    np.testing.assert_array_equal(np.argsort(keys, kind="stable"), np.argsort(skeys, kind="stable"))
    np.testing.assert_array_equal(td.skeys_to_keys(skeys), keys)
    assert skeys.max() == td.counts_to_skey(cs[1]) < td.SKEY_LIMIT <= 1 << _lib.TD_SKEY_BITS
    with pytest.raises(ValueError):
        td.counts_to_skey((10, 55) + (0,) * 8)
