"""libothello_cpu.so — include/othello.h built for the host over the oracle
("a CPU build of the same header gives identical results").

Called through the product's own ctypes signature table with host buffers and
checked against the golden fixtures from the real board.py; the GPU twin of
these calls is tests/test_gpu_abi_pair.py.  CPU only."""
import ctypes
import re
import subprocess

import numpy as np
import pytest

import oracle
from golden_io import ROLLOUT_FIXTURES, h, load_json, load_npz
from subproc_amd import _lib
from subproc_amd.td import skeys_to_keys

P = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


WORK = np.zeros(1, np.uint64)  # the rollouts' work word (unused by the host build, but required)


def lib():
    return oracle.cpu_abi()


def boards(black, white):
    return np.ascontiguousarray(np.stack([np.asarray(black, np.uint64), np.asarray(white, np.uint64)], 1))


def test_exports_every_header_symbol():
    from test_abi import header_functions
    lib()
    out = subprocess.run(["nm", "-D", "--defined-only", oracle.CPU_ABI_PATH], capture_output=True, text=True).stdout
    assert set(re.findall(r" T (oth_\w+)$", out, re.M)) == set(header_functions()) == set(_lib.SIGNATURES)
    assert lib().oth_version().decode().startswith("subproc_amd-cpu")


def test_reset_legal_step_opening():
    op = load_json("opening.json")
    b = np.zeros((4, 2), np.uint64)
    t = np.zeros(4, np.uint8)
    nt = np.full(4, 9, np.uint8)
    assert lib().oth_reset(P(b), P(t), P(nt), 4, None) == 0
    assert (b[:, 0] == h(op["black"])).all() and (b[:, 1] == h(op["white"])).all() and (t == 1).all()
    assert (nt == 0).all()
    leg = np.zeros(2, np.uint64)
    assert lib().oth_legal(P(b[:2].copy()), P(np.array([1, 2], np.uint8)), P(leg), 2, None) == 0
    assert leg[0] == h(op["legal_black"]) and leg[1] == h(op["legal_white"])


def test_step_every_code_midgame_fixture():
    z = load_npz("midgame_step.npz")
    n = len(z["black"])
    b = boards(z["black"], z["white"])
    for code in (0, 19, 26, 37, 44, 63, 64, 65, 200):
        bo = np.empty_like(b)
        to, ret, nt = np.empty(n, np.uint8), np.empty(n, np.int8), np.zeros(n, np.uint8)
        fl, ln = np.empty(n, np.uint64), np.empty(n, np.uint64)
        mv = np.full(n, code, np.uint8)
        assert lib().oth_step(P(b), P(z["turn"]), P(mv), P(bo), P(to), P(fl), P(ln), P(ret), P(nt), n, None) == 0
        if code <= 64:
            np.testing.assert_array_equal(ret, z["ret"][:, code])
            np.testing.assert_array_equal(bo[:, 0], z["next_black"][:, code])
            np.testing.assert_array_equal(bo[:, 1], z["next_white"][:, code])
            np.testing.assert_array_equal(to, z["next_turn"][:, code])
            np.testing.assert_array_equal(nt, z["next_nturn"][:, code])
            np.testing.assert_array_equal(ln, z["next_legal"][:, code])
        else:
            assert (ret == -1).all() and (bo == b).all()


@pytest.mark.parametrize("name", ROLLOUT_FIXTURES)
def test_rollout_fixtures(name):
    z = load_npz(name + ".npz")
    n = len(z["plies"])
    from_mid = "from_mid" in name
    st = boards(z["start_black"], z["start_white"]) if from_mid else None
    stt = z["start_turn"] if from_mid else None
    fb, df, pl = np.empty((n, 2), np.uint64), np.empty(n, np.int8), np.empty(n, np.uint8)
    mv, hist = np.empty((n, _lib.MOVES_STRIDE), np.uint8), np.zeros(_lib.HIST_BINS, np.int64)
    if "weights_white" in z:
        w = np.ascontiguousarray(z["weights"].reshape(-1), np.int8)
        ww = np.ascontiguousarray(z["weights_white"].reshape(-1), np.int8)
        rc = lib().oth_rollout_match(P(st), P(stt), int(z["seed"]), int(z["game_id0"]), int(z["n_random"]), P(w),
                                     P(ww), P(fb), P(df), P(pl), P(mv), P(hist), P(WORK), n, None)
    elif int(z["policy"]) == 2:
        w = np.ascontiguousarray(z["weights"].reshape(-1), np.int8)
        rc = lib().oth_rollout_eval(P(st), P(stt), int(z["seed"]), int(z["game_id0"]), int(z["n_random"]), P(w),
                                    P(fb), P(df), P(pl), P(mv), P(hist), P(WORK), n, None)
    else:
        rc = lib().oth_rollout(P(st), P(stt), int(z["seed"]), int(z["game_id0"]), int(z["policy"]),
                               int(z["n_random"]), P(fb), P(df), P(pl), P(mv), P(hist), P(WORK), n, None)
    assert rc == 0
    np.testing.assert_array_equal(mv, z["moves"])
    np.testing.assert_array_equal(fb[:, 0], z["final_black"])
    np.testing.assert_array_equal(fb[:, 1], z["final_white"])
    np.testing.assert_array_equal(df, z["diff"])
    np.testing.assert_array_equal(pl, z["plies"])
    assert hist[132] == int(z["plies"].astype(np.int64).sum())


def test_replay_and_book_text_fixture():
    """Books (§8f row 1): replay a fixture game, serialize every position."""
    bk = load_json("books.json")[0]
    z = load_npz(bk["source"] + ".npz")
    g = bk["game"]
    moves = np.ascontiguousarray(z["moves"][g:g + 1])
    plies = np.ascontiguousarray(z["plies"][g:g + 1])
    pos = np.zeros((1, _lib.POS_STRIDE, 2), np.uint64)
    pt, pe = np.zeros((1, _lib.POS_STRIDE), np.uint8), np.zeros((1, _lib.POS_STRIDE), np.uint8)
    assert lib().oth_replay(None, None, P(moves), P(plies), P(pos), P(pt), P(pe), 1, None) == 0
    k = int(plies[0]) + 1
    txt = np.zeros(k * _lib.BOOK_LINE, np.uint8)
    assert lib().oth_book_text(P(np.ascontiguousarray(pos[0, :k])), P(np.ascontiguousarray(pt[0, :k])), k,
                               P(txt), None) == 0
    assert txt.tobytes().decode().splitlines() == bk["lines"]
    assert [bool(e) for e in pe[0, :k]] == [r["end"] for r in bk["records"]]


def test_features_and_eval_fixture():
    z = load_npz("eval_values.npz")
    b = boards(z["black"], z["white"])
    n = len(b)
    for col, side in ((0, 1), (1, 2), (2, 0)):
        sd = np.full(n, side, np.uint8)
        f = np.empty((n, _lib.N_FEATURES), np.uint8)
        assert lib().oth_features(P(b), P(sd), P(f), n, None) == 0
        np.testing.assert_array_equal(f, z["counts"][:, col])
        for wk, ek in (("weights_default", "eval_default"), ("weights_rand", "eval_rand")):
            w = np.ascontiguousarray(z[wk].reshape(-1), np.int8)
            out = np.empty(n, np.int32)
            assert lib().oth_eval(P(b), P(sd), P(w), P(out), n, None) == 0
            np.testing.assert_array_equal(out, z[ek][:, col])


def test_sample_midgame_fixture_and_einval():
    z = load_npz("sample_midgame.npz")
    n = len(z["move"])
    b, t, nt, m = np.empty((n, 2), np.uint64), np.empty(n, np.uint8), np.empty(n, np.uint8), np.empty(n, np.uint8)
    assert lib().oth_sample_midgame(int(z["seed"]), 0, P(b), P(t), P(nt), P(m), n, None) == 0
    np.testing.assert_array_equal(b[:, 0], z["black"])
    np.testing.assert_array_equal(m, z["move"])
    assert lib().oth_rollout(None, None, 1, 0, 7, 0, None, None, None, None, None, P(WORK), 4, None) == _lib.OTH_EINVAL
    # the work word is required (include/othello.h)
    assert lib().oth_rollout(None, None, 1, 0, 0, 0, None, None, None, None, None, None, 4, None) == _lib.OTH_EINVAL
    assert lib().oth_step(None, None, None, None, None, None, None, None, None, 3, None) == _lib.OTH_EINVAL
    assert lib().oth_eval(None, None, None, None, 0, None) == _lib.OTH_EINVAL


@pytest.mark.parametrize("name", ["rollout_runner_eval", "rollout_runner_greedy", "rollout_runner_eval_mid"])
def test_rollout_runner_fixtures(name):
    z = load_npz(name + ".npz")
    n = len(z["plies"])
    st = boards(z["start_black"], z["start_white"])
    stt = np.ascontiguousarray(z["start_turn"])
    wa, wb = (ctypes.c_int8 * 36)(*z["weights_a"].reshape(-1).tolist()), (ctypes.c_int8 * 36)(*z["weights_b"].reshape(-1).tolist())
    fb, d, pl, ab = np.zeros((n, 2), np.uint64), np.zeros(n, np.int8), np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    mv, hist = np.zeros((n, 128), np.uint8), np.zeros(133, np.int64)
    rc = lib().oth_rollout_runner(P(st), P(stt), int(z["seed"]), int(z["game_id0"]), int(z["policy"]), wa, wb,
                                  int(z["n_rand_a"]), int(z["n_rand_b"]), int(z["swap"]), P(ab), P(fb), P(d), P(pl),
                                  P(mv), P(hist), P(WORK), n, None)
    assert rc == 0
    np.testing.assert_array_equal(mv, z["moves"])
    np.testing.assert_array_equal(ab, z["a_black"])
    np.testing.assert_array_equal(fb, boards(z["final_black"], z["final_white"]))
    assert int(hist[132]) == int(z["plies"].astype(np.int64).sum())
    E = _lib.OTH_EINVAL
    assert lib().oth_rollout_runner(None, None, 1, 0, 0, wa, wb, 0, 0, 0, None, None, None, None, None, None, P(WORK),
                                    4, None) == E  # random is not a runner policy
    assert lib().oth_rollout_runner(None, None, 1, 0, 2, None, wb, 0, 0, 0, None, None, None, None, None, None,
                                    P(WORK), 4, None) == E
    assert lib().oth_rollout_runner(None, None, 1, 0, 1, None, None, -1, 0, 0, None, None, None, None, None, None,
                                    P(WORK), 4, None) == E


def _scratch(fn, *args):
    tb = ctypes.c_size_t(0)
    assert fn(*args, None, ctypes.byref(tb), None) == 0
    temp = np.zeros(max(tb.value, 1), np.uint8)
    assert fn(*args, P(temp), ctypes.byref(tb), None) == 0


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


def test_td_sort_unpack_and_segments_words_host_build():
    """Round 5's oth_td_sort_unpack and oth_td_segments_words on the host build
    of the header, against numpy: the stable skey-bit order, the keys as
    OTH_TD_KEY values, the unpacked values, the runs of the sorted keys and the
    long ones."""
    rng = np.random.default_rng(3)
    n = 20000
    k = _skeys(rng, 300)[rng.integers(0, 300, n)].astype(np.uint64)  # repeats
    vs = rng.integers(-64, 65, n).astype(np.int64)
    tl = rng.integers(0, 129, n).astype(np.uint64)
    w = np.ascontiguousarray(((vs + 64).astype(np.uint64) << np.uint64(56)) | (tl << np.uint64(_lib.TD_PACK_TURN_SHIFT)) | k)
    lam = np.array([0.9 ** j for j in range(129)], np.float64)
    keys, vals = np.zeros(n, np.int64), np.zeros(n, np.float64)
    _scratch(lib().oth_td_sort_unpack, P(w), P(lam), P(keys), P(vals), n)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(keys, skeys_to_keys(k[order].astype(np.int64)))
    np.testing.assert_array_equal(vals, vs[order].astype(np.float64) * lam[tl[order].astype(np.int64)])
    sw = np.ascontiguousarray(w[order])
    off, uk, li, cnt, v2 = (np.zeros(n + 1, np.int64), np.zeros(n, np.int64), np.zeros(n, np.int64),
                            np.zeros(2, np.int64), np.zeros(n, np.float64))
    _scratch(lib().oth_td_segments_words, P(sw), P(lam), n, 48, P(off), P(uk), P(li), P(cnt), P(v2))
    np.testing.assert_array_equal(v2, vals)
    ks = skeys_to_keys(k[order].astype(np.int64))
    starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
    assert int(cnt[0]) == len(starts)
    np.testing.assert_array_equal(off[:len(starts) + 1], np.r_[starts, n])
    np.testing.assert_array_equal(uk[:len(starts)], ks[starts])
    want = np.flatnonzero(np.diff(np.r_[starts, n]) >= 48)
    assert int(cnt[1]) == len(want)
    np.testing.assert_array_equal(li[:len(want)], want)


def test_td_unpack_clamps_turn_left_host_build():
    """A packed word whose turn_left field exceeds 128 (not one
    oth_td_updates_packed writes) reads lam_pow[128], never past the table."""
    lam = np.array([0.9 ** j for j in range(129)], np.float64)
    tl = np.array([0, 128, 129, 0xFFFFF], np.uint64)
    w = np.ascontiguousarray((np.uint64(64 + 3) << np.uint64(56)) | (tl << np.uint64(_lib.TD_PACK_TURN_SHIFT)))
    keys, vals = np.zeros(4, np.int64), np.zeros(4, np.float64)
    cnt = ctypes.c_uint64(0)
    assert lib().oth_td_word_errors(ctypes.byref(cnt), 1, None) == 0
    assert lib().oth_td_unpack(P(w), P(lam), P(keys), P(vals), 4, None) == 0
    np.testing.assert_array_equal(vals, 3.0 * lam[[0, 128, 128, 128]])
    # the two words past the table are counted (oth_td_word_errors), not only clamped
    assert lib().oth_td_word_errors(ctypes.byref(cnt), 1, None) == 0 and cnt.value == 2
    assert lib().oth_td_word_errors(ctypes.byref(cnt), 0, None) == 0 and cnt.value == 0
