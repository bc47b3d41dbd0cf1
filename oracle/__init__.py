"""ctypes wrapper of the C parity oracle (oracle/othello_oracle.c).

TEST INFRASTRUCTURE ONLY — to be imported by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg as the *checker*; the product package
subproc_amd/ never imports it.  numpy in / numpy out, host memory only.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
CPU_ABI_PATH = os.path.join(_HERE, "libothello_cpu.so")
HIST_BINS = 133
MOVES_STRIDE = 128

_lib = None


def build(force=False):
    if force or not os.path.exists(LIB_PATH) or not os.path.exists(CPU_ABI_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE, "all"])


_cpu_abi = None


def cpu_abi():
    """libothello_cpu.so: include/othello.h on host memory, bound
    with the product's own signature table so both libraries are called alike."""
    global _cpu_abi
    if _cpu_abi is None:
        from subproc_amd._lib import SIGNATURES  # the table only; loads no GPU code
        if not os.path.exists(CPU_ABI_PATH):
            build()
        L = ctypes.CDLL(CPU_ABI_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _cpu_abi = L
    return _cpu_abi


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I64, U64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int
        L.oracle_reset.argtypes = [P, P, P, I64]
        L.oracle_legal.argtypes = [P, P, P, I64]
        L.oracle_step.argtypes = [P, P, P, P, P, P, P, P, P, I64]
        L.oracle_result.argtypes = [P, P, P, P, P, I64]
        L.oracle_rollout.argtypes = [P, P, U64, U64, I, I, P, P, P, P, P, I64, I, P, P]
        L.oracle_sample_midgame.argtypes = [U64, U64, P, P, P, P, I64]
        L.oracle_features.argtypes = [P, P, P, I64]
        L.oracle_eval.argtypes = [P, P, P, P, I64]
        L.oracle_replay.argtypes = [P, P, P, P, P, P, P, I64]
        L.oracle_hands.argtypes = [P, P, P, P, P, P, P, I64]
        L.oracle_rollout_ids.argtypes = [P, I64, U64, I, I, P, P, P, P, P]
        L.oracle_rollout_runner.argtypes = [P, P, U64, U64, I, P, P, I, I, I, P, P, P, P, P, P, I64, I]
        L.oracle_game_key.argtypes = [U64, U64]
        L.oracle_game_key.restype = U64
        L.oracle_rng_draws.argtypes = [U64, ctypes.c_uint32]
        L.oracle_rng_draws.restype = ctypes.c_uint32
        for f in ("oracle_reset", "oracle_legal", "oracle_step", "oracle_result", "oracle_rollout",
                  "oracle_sample_midgame", "oracle_features", "oracle_eval", "oracle_replay", "oracle_hands", "oracle_rollout_ids",
                  "oracle_rollout_runner"):
            getattr(L, f).restype = I
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _boards(b):
    b = np.ascontiguousarray(b, dtype=np.uint64)
    assert b.ndim == 2 and b.shape[1] == 2
    return b


def reset(n):
    b = np.empty((n, 2), np.uint64)
    t = np.empty(n, np.uint8)
    nt = np.empty(n, np.uint8)
    lib().oracle_reset(_p(b), _p(t), _p(nt), n)
    return b, t, nt


def legal(boards, turn):
    boards = _boards(boards)
    turn = np.ascontiguousarray(turn, np.uint8)
    out = np.empty(len(boards), np.uint64)
    lib().oracle_legal(_p(boards), _p(turn), _p(out), len(boards))
    return out


def step(boards, turn, move, nturn=None):
    boards = _boards(boards)
    n = len(boards)
    turn = np.ascontiguousarray(turn, np.uint8)
    move = np.ascontiguousarray(move, np.uint8)
    bo = np.empty((n, 2), np.uint64)
    to = np.empty(n, np.uint8)
    fl = np.empty(n, np.uint64)
    ln = np.empty(n, np.uint64)
    r = np.empty(n, np.int8)
    nt = None if nturn is None else np.array(nturn, np.uint8)
    lib().oracle_step(_p(boards), _p(turn), _p(move), _p(bo), _p(to), _p(fl), _p(ln), _p(r), _p(nt), n)
    return dict(boards=bo, turn=to, flips=fl, legal_next=ln, ret=r, nturn=nt)


def result(boards):
    boards = _boards(boards)
    n = len(boards)
    nb, nw, t = (np.empty(n, np.uint8) for _ in range(3))
    d = np.empty(n, np.int8)
    lib().oracle_result(_p(boards), _p(nb), _p(nw), _p(d), _p(t), n)
    return dict(n_black=nb, n_white=nw, diff=d, terminal=t)


def _weights(w):
    w = np.ascontiguousarray(np.asarray(w).reshape(-1))
    assert w.size == 36 and w.min() >= -128 and w.max() <= 127
    return w.astype(np.int8)


def rollout(n, seed, game_id0=0, policy=0, n_random=10, start=None, start_turn=None, record_moves=False,
            n_threads=0, weights=None, weights_white=None):
    """policy 0 random, 1 greedy, 2 eval (weights: 36 int8, [shard][feature];
    weights_white: White's table in a match, default = weights)."""
    w = None if weights is None else _weights(weights)
    ww = None if weights_white is None else _weights(weights_white)
    if policy == 2 and w is None:
        raise ValueError("policy 2 (eval) needs weights")
    start = None if start is None else _boards(start)
    st = None if start_turn is None else np.ascontiguousarray(start_turn, np.uint8)
    fb = np.empty((n, 2), np.uint64)
    d = np.empty(n, np.int8)
    pl = np.empty(n, np.uint8)
    mv = np.empty((n, MOVES_STRIDE), np.uint8) if record_moves else None
    h = np.zeros(HIST_BINS, np.int64)
    lib().oracle_rollout(_p(start), _p(st), seed, game_id0, policy, n_random, _p(fb), _p(d), _p(pl), _p(mv), _p(h),
                         n, n_threads, _p(w), _p(ww))
    return dict(final_boards=fb, diff=d, plies=pl, moves=mv, hist=h)


def rollout_runner(n, seed, game_id0=0, policy=2, weights_a=None, weights_b=None, n_rand_a=0, n_rand_b=0, swap=False,
                   start=None, start_turn=None, record_moves=False, n_threads=0):
    """GameRunner matches (include/othello.h oth_rollout_runner): player A vs
    player B, both greedy (1) or eval (2) with their own tables, GameRunner's
    random-move budgets and do_match's colour swap.  dict(..., a_black)."""
    wa = None if weights_a is None else _weights(weights_a)
    wb = None if weights_b is None else _weights(weights_b)
    start = None if start is None else _boards(start)
    st = None if start_turn is None else np.ascontiguousarray(start_turn, np.uint8)
    fb = np.empty((n, 2), np.uint64)
    d = np.empty(n, np.int8)
    pl = np.empty(n, np.uint8)
    ab = np.empty(n, np.uint8)
    mv = np.empty((n, MOVES_STRIDE), np.uint8) if record_moves else None
    h = np.zeros(HIST_BINS, np.int64)
    rc = lib().oracle_rollout_runner(_p(start), _p(st), seed, game_id0, policy, _p(wa), _p(wb), n_rand_a, n_rand_b,
                                     int(bool(swap)), _p(ab), _p(fb), _p(d), _p(pl), _p(mv), _p(h), n, n_threads)
    if rc != 0:
        raise ValueError("oracle_rollout_runner: invalid arguments")
    return dict(final_boards=fb, diff=d, plies=pl, moves=mv, hist=h, a_black=ab)


def rollout_ids(ids, seed, policy=0, n_random=10, weights=None, weights_white=None):
    """The games of global ids `ids` (any order / stride) from the opening, as
    oracle_rollout plays them: dict(final_boards, diff, plies)."""
    ids = np.ascontiguousarray(ids, np.uint64)
    n = len(ids)
    w = None if weights is None else _weights(weights)
    ww = None if weights_white is None else _weights(weights_white)
    fb = np.empty((n, 2), np.uint64)
    d = np.empty(n, np.int8)
    pl = np.empty(n, np.uint8)
    rc = lib().oracle_rollout_ids(_p(ids), n, seed, policy, n_random, _p(w), _p(ww), _p(fb), _p(d), _p(pl))
    assert rc == 0
    return dict(final_boards=fb, diff=d, plies=pl)


def sample_midgame(n, seed, index0=0):
    b = np.empty((n, 2), np.uint64)
    t, nt, m = (np.empty(n, np.uint8) for _ in range(3))
    lib().oracle_sample_midgame(seed, index0, _p(b), _p(t), _p(nt), _p(m), n)
    return dict(boards=b, turn=t, nturn=nt, move=m)


def features(boards, side):
    boards = _boards(boards)
    side = np.ascontiguousarray(side, np.uint8)
    out = np.empty((len(boards), 10), np.uint8)
    lib().oracle_features(_p(boards), _p(side), _p(out), len(boards))
    return out


def evaluate(boards, side, weights):
    boards = _boards(boards)
    side = np.ascontiguousarray(side, np.uint8)
    out = np.empty(len(boards), np.int32)
    lib().oracle_eval(_p(boards), _p(side), _p(_weights(weights)), _p(out), len(boards))
    return out


def replay(moves, plies, start=None, start_turn=None):
    moves = np.ascontiguousarray(moves, np.uint8)
    plies = np.ascontiguousarray(plies, np.uint8)
    n = len(plies)
    start = None if start is None else _boards(start)
    st = None if start_turn is None else np.ascontiguousarray(start_turn, np.uint8)
    pos = np.zeros((n, MOVES_STRIDE + 1, 2), np.uint64)
    t = np.zeros((n, MOVES_STRIDE + 1), np.uint8)
    e = np.zeros((n, MOVES_STRIDE + 1), np.uint8)
    lib().oracle_replay(_p(start), _p(st), _p(moves), _p(plies), _p(pos), _p(t), _p(e), n)
    return dict(boards=pos, turn=t, end=e)


def hands(boards, piece, x, y, dx, dy):
    """len(hands_for_direc((dx, dy), piece, x, y)) per item (board.py:124-139):
    piece any 0..255, origin and direction any int64.  (n,) uint8."""
    boards = _boards(boards)
    n = len(boards)
    piece = np.ascontiguousarray(np.broadcast_to(piece, n), np.uint8)
    x, y, dx, dy = (np.ascontiguousarray(np.broadcast_to(v, n), np.int64) for v in (x, y, dx, dy))
    out = np.empty(n, np.uint8)
    lib().oracle_hands(_p(boards), _p(piece), _p(x), _p(y), _p(dx), _p(dy), _p(out), n)
    return out


def serialize_str(black, white, turn):
    """board.py:214-243 restated for the checker (row-major, O = Black, X = White)."""
    black, white = int(black), int(white)
    b = "".join("O" if black >> i & 1 else "X" if white >> i & 1 else "-" for i in range(64))
    return b + " " + ("O" if turn == 1 else "X" if turn == 2 else "-")


def game_key(seed, g):
    return lib().oracle_game_key(seed, g)


def rng_draw(key, i):
    """The i-th (1-based) draw of game key `key`'s LCG stream."""
    return lib().oracle_rng_draws(key, i)


def td_state_map(pos_boards, plies, store=None, a=0.03, lam=0.90):
    """progress_position_moves_learn.py:37-62 restated over the oracle's counts():
    books = games in order, each walked terminal -> opening, sides 'O' then 'X'.
    pos_boards (n, 129, 2) uint64 replay rows, plies (n,).  Returns {counts tuple:
    value} (pure-Python EMA loop: small cases only)."""
    store = {} if store is None else store
    pos_boards = np.asarray(pos_boards, np.uint64)
    n = len(plies)
    for g in range(n):
        np_ = min(int(plies[g]), MOVES_STRIDE)
        rows = np.ascontiguousarray(pos_boards[g, :np_ + 1])
        fb = features(rows, np.full(np_ + 1, 1, np.uint8))
        fw = features(rows, np.full(np_ + 1, 2, np.uint8))
        term = rows[np_]
        vb = bin(int(term[0])).count("1") - bin(int(term[1])).count("1")
        for p in range(np_, -1, -1):
            for f, value in ((fb[p], vb), (fw[p], -vb)):
                key = tuple(int(x) for x in f)
                cur = float(store.get(key, 0))
                new = float(value) * (lam ** (np_ - p))
                store[key] = new if cur == 0 else cur * (1 - a) + new * a
    return store
