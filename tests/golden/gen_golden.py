#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REAL reference board.py.

TEST INFRASTRUCTURE ONLY.  Runs in the build container only (never on the GPU
box): it needs /root/reference/board.py and refuses to run without it.

How the reference is loaded: board.py is Python 2 but only two
lines are not valid Python 3, so its text is read, exactly two substitutions are
applied in memory, and the result is exec'd into a private namespace:
  * board.py:92  ``print q``  -> ``print(q)``      (display-only show_mask)
  * board.py:257 ``i / 8``    -> ``i // 8``        (deserialize row index)
Nothing is written to /root/reference and no reference source is copied into
this repository; only inputs/outputs (data) are committed.

The move-selection rule for rollouts is OUR spec (board.py has no RNG; the
reference picks with Python's ``random.randrange`` in game_runner.py:133-152).
The spec is restated here in pure Python and every trajectory is driven through
board.py's own ``puttables`` / ``put_s`` / ``is_game_over`` so the fixtures pin
(board, move) -> next state semantics to the reference, and the RNG spec to a
second independent implementation.

Usage:  python tests/golden/gen_golden.py [--out DIR]   (all 24 fixtures, ≈1–2 min on 8 cores)
        python tests/golden/gen_golden.py --only batch_stats|td_records|runner|board_api
"""
import json
import random
import multiprocessing as mp
import os
import sys

import numpy as np

REF = "/root/reference/board.py"
OUT = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1
M32 = (1 << 32) - 1
GOLDEN64 = 0x9E3779B97F4A7C15
PASS = 64
SEED = 0x5EED


# ----------------------------------------------------------------------------
# reference loader (the shim of SURVEY.md §8c)
# ----------------------------------------------------------------------------
def load_reference_board():
    if not os.path.exists(REF):
        sys.exit("gen_golden.py: /root/reference/board.py absent - fixtures can only be generated in the build container")
    src = open(REF).read()
    a, b = "        print q\n", "i % 8, i / 8)"
    assert src.count(a) == 1 and src.count(b) == 1, "board.py changed; shim substitutions no longer apply"
    src = src.replace(a, "        print(q)\n").replace(b, "i % 8, i // 8)")
    ns = {"__name__": "reference_board"}
    exec(compile(src, "reference_board.py", "exec"), ns)
    return ns


RB = load_reference_board()
Board = RB["Board"]


def load_reference_counts(want_ns=False):
    """parameter_progress_position_moves_learn.counts (and parameter.board_from_a_book)
    from the reference, exec'd against the shimmed board module.  Both files are
    valid Python 3 as they stand; nothing is copied.  want_ns=True returns the
    module namespace (for ProgressPositionMovesParameter.default_value)."""
    import types
    mod_board = types.ModuleType("board")
    mod_board.__dict__.update(RB)
    saved = {k: sys.modules.get(k) for k in ("board", "parameter")}
    sys.modules["board"] = mod_board
    try:
        mod_param = types.ModuleType("parameter")
        exec(compile(open("/root/reference/parameter.py").read(), "reference_parameter.py", "exec"),
             mod_param.__dict__)
        sys.modules["parameter"] = mod_param
        ns = {"__name__": "reference_ppml"}
        exec(compile(open("/root/reference/parameter_progress_position_moves_learn.py").read(),
                     "reference_ppml.py", "exec"), ns)
        return ns if want_ns else ns["counts"]
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
Black, White, Empty = RB["Black"], RB["White"], RB["Empty"]


# ----------------------------------------------------------------------------
# helpers: reference Board <-> bitboards (sq = x + 8*y, SURVEY.md §8 conventions)
# ----------------------------------------------------------------------------
def to_bits(b):
    bl = wh = 0
    for y in range(8):
        for x in range(8):
            c = b.get(x, y)
            if c == Black:
                bl |= 1 << (x + 8 * y)
            elif c == White:
                wh |= 1 << (x + 8 * y)
    return bl, wh


def from_bits(bl, wh, turn, nturn=0):
    b = Board()
    for y in range(8):
        for x in range(8):
            sq = x + 8 * y
            b.set(Black if bl >> sq & 1 else White if wh >> sq & 1 else Empty, x, y)
    b.turn = turn
    b.nturn = nturn
    return b


def clone(b):
    c = Board()
    c.board = [row[:] for row in b.board]
    c.turn, c.nturn = b.turn, b.nturn
    return c


def legal_bits(b, piece):
    m = 0
    for (x, y) in b.puttables(piece):
        m |= 1 << (x + 8 * y)
    return m


def code_to_str(b, code):
    return "ps" if code == PASS else b.handstr_from_coord(code % 8, code // 8)


def hostile(t):
    return White if t == Black else Black


# ----------------------------------------------------------------------------
# RNG spec — pure-Python restatement
# ----------------------------------------------------------------------------
def mix64(z):
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def mix32(x):
    x &= M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


LCG_MUL = 0x915F77F5  # 32-bit LCG multiplier (Steele & Vigna 2021 tables)


def seed_state(seed):
    return mix64((seed + GOLDEN64) & M64)


def game_key(S, g):
    return mix64((S + g * GOLDEN64) & M64)


class GameRng:
    """Per-game draw stream: state0 = lo32(key), increment = hi32(key) | 1;
    each draw advances state = state * LCG_MUL + inc (mod 2^32) and returns it.
    A uniform pick in [0, n) is (draw * n) >> 32."""

    def __init__(self, key):
        self.state = key & M32
        self.inc = (key >> 32) | 1

    def draw(self):
        self.state = (self.state * LCG_MUL + self.inc) & M32
        return self.state

    def pick(self, n):
        return (self.draw() * n) >> 32


# ----------------------------------------------------------------------------
# trajectories driven through board.py
# ----------------------------------------------------------------------------
def play(args):
    """One game from (bl, wh, turn) to terminal via board.py.

    policy 0 = random (k-th legal square, LSB-first == puttables order);
    policy 1 = greedy: for ply >= n_random pick the legal move minimising the
    opponent's n_puttable_for on the child, ties -> first in puttables order.
    policy 2 = eval: for ply >= n_random pick the legal move maximising the
    mover's linear eval of the child (eval_value: the reference's own counts()
    on the child's book record), ties -> first in puttables order.
    A side with no legal move passes ('ps'), as the engines do in game_runner.
    """
    seed, g, policy, n_random, bl, wh, turn = args[:7]
    weights = args[7] if len(args) > 7 else None
    weights_white = args[8] if len(args) > 8 and args[8] is not None else weights  # a match: White's table
    rng = GameRng(game_key(seed_state(seed), g))
    b = from_bits(bl, wh, turn)
    moves = []
    ply = 0
    while not b.is_game_over():
        puts = b.puttables(b.turn)
        if not puts:
            code = PASS
        elif policy == 0 or ply < n_random:
            x, y = puts[rng.pick(len(puts))]
            code = x + 8 * y
        elif policy == 1:
            best, bestv = None, None
            for (x, y) in puts:
                c = clone(b)
                assert c.put_s(c.handstr_from_coord(x, y)) > 0
                v = c.n_puttable_for(hostile(b.turn))
                if bestv is None or v < bestv:
                    best, bestv = x + 8 * y, v
            code = best
        else:
            best, bestv = None, None
            for (x, y) in puts:
                c = clone(b)
                assert c.put_s(c.handstr_from_coord(x, y)) > 0
                v = eval_value(c, "O" if b.turn == Black else "X", weights if b.turn == Black else weights_white)
                if bestv is None or v > bestv:
                    best, bestv = x + 8 * y, v
            code = best
        r = b.put_s(code_to_str(b, code))
        assert r >= 0
        moves.append(code)
        ply += 1
    fb, fw = to_bits(b)
    return moves, fb, fw, b.n_black() - b.n_white(), ply


def policy_move(b, policy, weights):
    """The 1-ply policies of play() for the side to move (a legal move exists)."""
    best, bestv = None, None
    for (x, y) in b.puttables(b.turn):
        c = clone(b)
        assert c.put_s(c.handstr_from_coord(x, y)) > 0
        if policy == 1:
            v = -c.n_puttable_for(hostile(b.turn))
        else:
            v = eval_value(c, "O" if b.turn == Black else "X", weights)
        if bestv is None or v > bestv:
            best, bestv = x + 8 * y, v
    return best


def play_runner(args):
    """One GameRunner match (game_runner.py:104-201 as subproc.do_match runs
    it, subproc.py:15-39) between player A and player B, both playing
    `policy` (1 greedy, 2 eval with their own tables), driven through board.py.
    The reference draws with Python's random; here the same decisions draw
    from the game's counter stream, in the same order:
      * do_match: with randomize_black_white, randrange(2) == 1 swaps A and B
        (A then plays White) -> pick(2) == 1;
      * GameRunner.__init__: n_rand_rest = min(n_rand_hands, N_RAND_HAND_UNTIL);
      * go_for, on every turn of a player with n_rand_rest > 0 (passes
        included): randrange(n_rand_rest) == 0 -> pick(r) == 0; then if
        puttables is not empty, puttables[randrange(len)] -> pick(len) and
        n_rand_rest -= 1; otherwise the engine's own move (the policy), or PS.
    """
    seed, g, policy, wa, wb, n_rand_a, n_rand_b, swap, bl, wh, turn = args
    rng = GameRng(game_key(seed_state(seed), g))
    a_black = not (swap and rng.pick(2) == 1)
    ra, rb = min(n_rand_a, 10), min(n_rand_b, 10)
    players = {Black: {"w": wa if a_black else wb, "rest": ra if a_black else rb},
               White: {"w": wb if a_black else wa, "rest": rb if a_black else ra}}
    b = from_bits(bl, wh, turn)
    moves = []
    while not b.is_game_over():
        pl = players[b.turn]
        code = None
        if pl["rest"] > 0 and rng.pick(pl["rest"]) == 0:
            puts = b.puttables(b.turn)
            if len(puts) > 0:
                x, y = puts[rng.pick(len(puts))]
                code = x + 8 * y
                pl["rest"] -= 1
        if code is None:
            code = policy_move(b, policy, pl["w"]) if b.puttables(b.turn) else PASS
        assert b.put_s(code_to_str(b, code)) >= 0
        moves.append(code)
    fb, fw = to_bits(b)
    return moves, fb, fw, b.n_black() - b.n_white(), len(moves), int(a_black)


def runner_fixtures(pool):
    """rollout_runner_*.npz: GameRunner matches (play_runner) through board.py."""
    ib, iw = to_bits(Board())
    ns = load_reference_counts(want_ns=True)
    wdef = [list(r) for r in ns["ProgressPositionMovesParameter"]().default_value()]
    wrand = np.random.default_rng(77).integers(-127, 128, (4, 9)).tolist()
    mid = [(p[0], p[1], p[2]) for p in random_positions(256, 20240601) if p[2] in (Black, White)][:48]

    def runner(name, seed, g0, n, policy, wa, wb, n_rand_a, n_rand_b, swap, starts=None):
        starts = starts or [(ib, iw, Black)] * n
        args = [(seed, g0 + i, policy, wa, wb, n_rand_a, n_rand_b, swap, *st) for i, st in enumerate(starts)]
        res = pool.map(play_runner, args, chunksize=4)
        mv = np.full((n, 128), 255, np.uint8)
        for i, r in enumerate(res):
            mv[i, :len(r[0])] = r[0]
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"),
            seed=np.array(seed, np.uint64), game_id0=np.array(g0, np.uint64), policy=np.array(policy),
            n_rand_a=np.array(n_rand_a), n_rand_b=np.array(n_rand_b), swap=np.array(int(swap)),
            start_black=u64([s[0] for s in starts]), start_white=u64([s[1] for s in starts]),
            start_turn=np.array([s[2] for s in starts], np.uint8),
            moves=mv, final_black=u64([r[1] for r in res]), final_white=u64([r[2] for r in res]),
            diff=np.array([r[3] for r in res], np.int8), plies=np.array([r[4] for r in res], np.uint8),
            a_black=np.array([r[5] for r in res], np.uint8),
            weights_a=np.array(wa if wa is not None else [[0] * 9] * 4, np.int8),
            weights_b=np.array(wb if wb is not None else [[0] * 9] * 4, np.int8))

    runner("rollout_runner_eval", 6161, 40, 128, 2, wdef, wrand, 10, 3, True)
    runner("rollout_runner_greedy", 6262, 1 << 33, 96, 1, None, None, 4, 0, False)
    runner("rollout_runner_eval_mid", 6363, 7, len(mid), 2, wrand, wdef, 25, 7, True, starts=mid)


# learner shards of the disc count (ProgressPositionMovesLearn.__get_fit_parameters_shards,
# progress_position_moves_learn.py:112-113; that module needs pyres/slack, so the
# four bounds are restated here)
EVAL_SHARDS = ((0, 16), (17, 32), (33, 48), (49, 64))
_COUNTS = None


def eval_value(b, side, weights):
    """The learner's linear model on a board: sum_j W[shard(counts[0])][j] * counts[1+j]
    with the reference's counts() (fit in progress_position_moves_learn.py:160-184)."""
    global _COUNTS
    if _COUNTS is None:
        _COUNTS = load_reference_counts()
    f = _COUNTS({"book": b.serialize_board(), "whosturn": b.serialize_turn(), "turn": b.nturn}, side)
    k = [i for i, (lo, hi) in enumerate(EVAL_SHARDS) if lo <= f[0] <= hi][0]
    return sum(int(weights[k][j]) * int(f[1 + j]) for j in range(9))


def sample_midgame(args):
    """Config-2 input generator spec: see DESIGN.md §Synthetic mid-game positions."""
    seed, i = args
    S = seed_state(seed)
    attempt = 0
    while True:
        g = i ^ (attempt << 48)
        rng = GameRng(game_key(S, g))
        target = 10 + rng.pick(40)  # the first draw picks the stopping ply
        b = Board()
        ply = 0
        ok = False
        while not b.is_game_over():
            puts = b.puttables(b.turn)
            if ply >= target and puts:
                ok = True
                break
            if not puts:
                code = PASS
            else:
                x, y = puts[rng.pick(len(puts))]
                code = x + 8 * y
            assert b.put_s(code_to_str(b, code)) >= 0
            ply += 1
        if ok:
            puts = b.puttables(b.turn)
            x, y = puts[rng.pick(len(puts))]
            bl, wh = to_bits(b)
            return bl, wh, b.turn, ply, x + 8 * y
        attempt += 1


def step_all_codes(args):
    """For one position: every move code 0..64 through board.put_s (board.py:192-209)."""
    bl, wh, turn = args
    b0 = from_bits(bl, wh, turn)
    out = []
    for code in range(65):
        b = clone(b0)
        r = b.put_s(code_to_str(b, code))
        nb, nw = to_bits(b)
        out.append((r, nb, nw, b.turn, b.nturn, legal_bits(b, b.turn)))
    return legal_bits(b0, turn), out


def random_positions(n, seed):
    """Reachable positions for the step fixture: random play (python random, any
    reachable position will do) stopped at a uniformly random ply; includes
    positions where the mover must pass and terminal positions."""
    import random
    rnd = random.Random(seed)
    pos = []
    while len(pos) < n:
        b = Board()
        stop = rnd.randrange(0, 70)
        ply = 0
        while ply < stop and not b.is_game_over():
            puts = b.puttables(b.turn)
            s = "ps" if not puts else b.handstr_from_coord(*puts[rnd.randrange(len(puts))])
            b.put_s(s)
            ply += 1
        bl, wh = to_bits(b)
        pos.append((bl, wh, b.turn))
    return pos


def u64(a):
    return np.array(a, dtype=np.uint64)


# ----------------------------------------------------------------------------
# board_api: the inputs board.py accepts beyond Black/White play (round 2)
# ----------------------------------------------------------------------------
OTHER = 3  # a piece / side value equal to none of Empty, Black, White
API_PIECES = (Empty, Black, White, OTHER)
API_XY = tuple(range(-8, 8))       # what board[y][x] accepts (negatives wrap)
SCAN_XY = tuple(range(-3, 11))     # hands_for_direc takes any origin
SCAN_DIRECS = list(RB["DIRECS"]) + [(0, 0), (2, 1), (-1, 3)]


def api_boards(pos):
    """Positions for the piece/coordinate fixtures: reachable mid-game boards
    plus boards built to hit the unusual branches -- full rows/diagonals (a
    run of 8 hostile squares from an off-board origin), the wrapped origin on
    a later ray of put, and Black runs ending on empty squares."""
    out = [(p[0], p[1]) for p in pos[:24]]
    out += [
        (0, 0xFF),                                   # row 1 all White
        (0xFF, 0),                                   # row 1 all Black
        (0x8040201008040201, 0),                     # a1-h8 diagonal Black
        (0, 0x0102040810204080),                     # h1-a8 diagonal White
        (0x0000000000020000, 0x0000007F01000000),    # put(Black, -1, 4): RU, then R through the wrapped h5
        (0x0000007F00000000, 0x0000000000080000),    # Black row e..: runs ending on empties
        (0x00FF00000000FF00, 0x0000FF0000FF0000),
        (0x0101010101010101, 0x8080808080808080),    # files a / h full
    ]
    return out


def api_record(args):
    """For one board: put / is_puttable_at for every piece and (x, y) in
    -8..7, puttables for every piece, hands_for_direc lengths for SCAN_XY x
    SCAN_DIRECS, through board.py itself."""
    bl, wh = args
    b0 = from_bits(bl, wh, Black)
    n_xy = len(API_XY)
    put_ret = np.zeros((len(API_PIECES), n_xy, n_xy), np.int8)
    put_black = np.zeros((len(API_PIECES), n_xy, n_xy), np.uint64)
    put_white = np.zeros((len(API_PIECES), n_xy, n_xy), np.uint64)
    puttable = np.zeros((len(API_PIECES), n_xy, n_xy), np.uint8)
    legal = np.zeros(len(API_PIECES), np.uint64)
    hands = np.zeros((len(API_PIECES), len(SCAN_DIRECS), len(SCAN_XY), len(SCAN_XY)), np.uint8)
    for pi, piece in enumerate(API_PIECES):
        legal[pi] = legal_bits(b0, piece)
        for iy, y in enumerate(API_XY):
            for ix, x in enumerate(API_XY):
                puttable[pi, iy, ix] = b0.is_puttable_at(piece, x, y)
                b = clone(b0)
                put_ret[pi, iy, ix] = b.put(piece, x, y)
                assert all(c in (Empty, Black, White) for row in b.board for c in row)
                put_black[pi, iy, ix], put_white[pi, iy, ix] = to_bits(b)
        for di, d in enumerate(SCAN_DIRECS):
            for iy, y in enumerate(SCAN_XY):
                for ix, x in enumerate(SCAN_XY):
                    hs = b0.hands_for_direc(d, piece, x, y)
                    assert hs == [(piece, x + i * d[0], y + i * d[1]) for i in range(1, len(hs) + 1)]
                    hands[pi, di, iy, ix] = len(hs)
    return legal, puttable, put_ret, put_black, put_white, hands


def side_steps(args):
    """Every code 0..64 through put_s with the side to move `turn` (Empty via
    deserialize(..., '-', n), or a value no square holds), board.py:192-209."""
    bl, wh, turn = args
    b0 = from_bits(bl, wh, Black)
    if turn == Empty:
        b0.deserialize(b0.serialize_board(), "-", 7)
        assert b0.turn == Empty
    else:
        b0.turn, b0.nturn = turn, 7
    out = []
    for code in range(65):
        b = clone(b0)
        r = b.put_s(code_to_str(b, code))
        nb, nw = to_bits(b)
        out.append((r, nb, nw, b.turn, b.nturn, legal_bits(b, b.turn)))
    return legal_bits(b0, b0.turn), out


def board_api_fixtures(pos, pool):
    boards = api_boards(pos)
    res = pool.map(api_record, boards, chunksize=1)
    np.savez_compressed(
        os.path.join(OUT, "board_api.npz"),
        black=u64([b[0] for b in boards]), white=u64([b[1] for b in boards]),
        pieces=np.array(API_PIECES, np.uint8), xy=np.array(API_XY, np.int64), scan_xy=np.array(SCAN_XY, np.int64),
        scan_direcs=np.array(SCAN_DIRECS, np.int64),
        legal=np.stack([r[0] for r in res]), puttable=np.stack([r[1] for r in res]),
        put_ret=np.stack([r[2] for r in res]), put_black=np.stack([r[3] for r in res]),
        put_white=np.stack([r[4] for r in res]), hands=np.stack([r[5] for r in res]))
    # side to move Empty / other: every code
    cases = [(p[0], p[1], t) for t in (Empty, OTHER) for p in pos[:256]]
    res = pool.map(side_steps, cases, chunksize=8)
    np.savez_compressed(
        os.path.join(OUT, "side_steps.npz"),
        black=u64([c[0] for c in cases]), white=u64([c[1] for c in cases]),
        turn=np.array([c[2] for c in cases], np.uint8), legal=u64([r[0] for r in res]),
        ret=np.array([[o[0] for o in r[1]] for r in res], np.int8),
        next_black=u64([[o[1] for o in r[1]] for r in res]), next_white=u64([[o[2] for o in r[1]] for r in res]),
        next_turn=np.array([[o[3] for o in r[1]] for r in res], np.uint8),
        next_nturn=np.array([[o[4] for o in r[1]] for r in res], np.uint8),
        next_legal=u64([[o[5] for o in r[1]] for r in res]))
    # the live board list, other-valued cells and deserialize edge cases (JSON)
    recs = []
    for name, ops_ in [
        ("write_through", [("board", 2, 3, White), ("board", 4, 4, Empty), ("set", Black, -1, -1),
                           ("set", White, 0, -8)]),
        ("other_values", [("set", 5, 2, 3), ("set", 5, 5, 4), ("set", "x", -3, -2)]),
        ("other_blocks_run", [("set", 7, 5, 3), ("board", 3, 5, 7)]),
    ]:
        b = Board()
        for op in ops_:
            if op[0] == "board":
                b.board[op[1]][op[2]] = op[3]
            else:
                b.set(op[1], op[2], op[3])
        rec = {"name": name, "ops": [list(o) for o in ops_],
               "cells": [[c if isinstance(c, int) else str(c) for c in row] for row in b.board],
               "n_black": b.n_black(), "n_white": b.n_white(), "n_empty": b.n_empty(),
               "is_game_over": b.is_game_over(), "serialize_str": b.serialize_str(), "str": str(b),
               "puttables": {str(p): b.puttables(p) for p in (Empty, Black, White, 5, 7)},
               "mask_count": {str(p): b.mask_count(p, 0x00FFFF0000FFFF00) for p in (Empty, Black, White, 5, 7)},
               "get": [b.get(x, y) if isinstance(b.get(x, y), int) else str(b.get(x, y))
                       for (x, y) in ((-1, -1), (3, 2), (-5, -6), (2, 3))],
               "put_s": []}
        for code in range(65):
            c = clone(b)
            r = c.put_s(code_to_str(c, code))
            rec["put_s"].append({"code": code, "ret": r, "turn": c.turn,
                                 "cells": [[v if isinstance(v, int) else str(v) for v in row] for row in c.board]})
        rec["put"] = []
        for piece in (Empty, Black, White, 5, 7):
            for (x, y) in ((2, 2), (-1, 4), (3, 3), (5, 2), (0, -1), (4, 2)):
                c = clone(b)
                r = c.put(piece, x, y)
                rec["put"].append({"piece": piece, "x": x, "y": y, "ret": r,
                                   "cells": [[v if isinstance(v, int) else str(v) for v in row] for row in c.board]})
        recs.append(rec)
    dz = []
    for bstr, tstr in (("O" * 70, "X"), ("-" * 10, "O"), ("XO" * 32, "?")):
        b = Board()
        try:
            b.deserialize(bstr, tstr, 3)
            raised = False
        except IndexError:
            raised = True
        dz.append({"board": bstr, "turn_str": tstr, "raises": raised, "cells": [list(r) for r in b.board],
                   "turn": b.turn, "nturn": b.nturn})
    json.dump({"boards": recs, "deserialize": dz}, open(os.path.join(OUT, "board_api.json"), "w"))


def main():
    pool = mp.Pool(8)
    init = Board()
    ib, iw = to_bits(init)
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "board_api":
        board_api_fixtures(random_positions(1024, 20240601), pool)
        print("board_api fixtures written to", OUT)
        return

    # ---------------------------------------------------------------- opening
    opening = {"black": hex(ib), "white": hex(iw), "turn": init.turn, "nturn": init.nturn,
               "legal_black": hex(legal_bits(init, Black)), "legal_white": hex(legal_bits(init, White)),
               "is_game_over": init.is_game_over(), "moves": []}
    for (x, y) in init.puttables(init.turn):
        b = clone(init)
        s = b.handstr_from_coord(x, y)
        r = b.put_s(s)
        nb, nw = to_bits(b)
        opening["moves"].append({"move": s, "sq": x + 8 * y, "ret": r, "flips": hex(iw & ~nw),
                                 "black": hex(nb), "white": hex(nw), "turn": b.turn, "nturn": b.nturn})
    opening["strings"] = []
    for s in ["d4", "a1", "ps", "PS", "Ps", "xyz", "a0", "D3", "Bd3", "Wc4", "BWf5", "e6 ", "", "  c4", "h8", "9a1", "x-1"]:
        b = clone(init)
        r = b.put_s(s)
        nb, nw = to_bits(b)
        opening["strings"].append({"s": s, "ret": r, "black": hex(nb), "white": hex(nw),
                                   "turn": b.turn, "nturn": b.nturn})
    opening["index_error"] = []
    for s in ["a9", "i1", "z1", "zz9"]:
        b = clone(init)
        try:
            b.put_s(s)
            opening["index_error"].append({"s": s, "raises": False})
        except IndexError:
            opening["index_error"].append({"s": s, "raises": True})
    # codecs on the opening
    opening["serialize_str"] = init.serialize_str()
    opening["serialize_board"] = init.serialize_board()
    opening["str"] = str(init)
    json.dump(opening, open(os.path.join(OUT, "opening.json"), "w"), indent=1)

    # ---------------------------------------------------------------- edges
    edges = []

    def edge(name, bl, wh, turn, codes=tuple(range(65))):
        b0 = from_bits(bl, wh, turn)
        rec = {"name": name, "black": hex(bl), "white": hex(wh), "turn": turn,
               "is_game_over": b0.is_game_over(), "n_black": b0.n_black(), "n_white": b0.n_white(),
               "n_empty": b0.n_empty(), "legal_black": hex(legal_bits(b0, Black)),
               "legal_white": hex(legal_bits(b0, White)), "serialize_str": b0.serialize_str(), "steps": []}
        for code in codes:
            b = clone(b0)
            r = b.put_s(code_to_str(b, code))
            nb, nw = to_bits(b)
            rec["steps"].append({"code": code, "ret": r, "black": hex(nb), "white": hex(nw), "turn": b.turn})
        edges.append(rec)

    full = (1 << 64) - 1
    edge("full_board_black_wins", full & ~0xFF, 0xFF, Black)
    edge("full_board_draw", 0x00000000FFFFFFFF, 0xFFFFFFFF00000000, White)
    edge("wipeout_white_gone", 0x0000001818000000, 0, White)
    edge("wipeout_black_gone", 0, 0x0000001818000000, Black)
    edge("empty_board", 0, 0, Black)
    # mover (Black) has no move, White has: black a1, white b1, c1 empty..  Black: a1; White: b1 -> white can't move? construct:
    # Black at a1 only, White at b1,c1; Black to move: d1 flips b1,c1 -> legal; instead use Black on h8 isolated
    edge("mover_has_none_opponent_has", 1 << 0, (1 << 1), White)  # white to move: W b1 next to B a1 -> W has no flank; B has c1
    edge("pass_with_moves_available", ib, iw, Black, codes=(64, 19, 0))
    edge("long_ray_h_flip", 0x01, 0x7E, Black)  # b1..g1 white, a1 black: h1 flips six
    edge("diag_and_vertical", (1 << 0) | (1 << 7) | (1 << 56), 0x0040201008040200 | (0x0001010101010100 & ~1), Black)
    edge("corner_multi_dir", 0x8100000000000081, 0x42C300000000C342, Black)
    json.dump(edges, open(os.path.join(OUT, "edges.json"), "w"), indent=1)

    # ---------------------------------------------------------------- step, every code
    pos = random_positions(1024, 20240601)
    res = pool.map(step_all_codes, pos, chunksize=8)
    np.savez_compressed(
        os.path.join(OUT, "midgame_step.npz"),
        black=u64([p[0] for p in pos]), white=u64([p[1] for p in pos]),
        turn=np.array([p[2] for p in pos], np.uint8),
        legal=u64([r[0] for r in res]),
        ret=np.array([[o[0] for o in r[1]] for r in res], np.int8),
        next_black=u64([[o[1] for o in r[1]] for r in res]),
        next_white=u64([[o[2] for o in r[1]] for r in res]),
        next_turn=np.array([[o[3] for o in r[1]] for r in res], np.uint8),
        next_nturn=np.array([[o[4] for o in r[1]] for r in res], np.uint8),
        next_legal=u64([[o[5] for o in r[1]] for r in res]),
    )

    board_api_fixtures(pos, pool)

    # ---------------------------------------------------------------- rollouts
    def rollouts(name, seed, g0, n, policy, n_random, starts=None, weights=None, weights_white=None):
        if starts is None:
            starts = [(ib, iw, Black)] * n
        args = [(seed, g0 + i, policy, n_random, s[0], s[1], s[2], weights, weights_white)
                for i, s in enumerate(starts)]
        res = pool.map(play, args, chunksize=4)
        mv = np.full((n, 128), 255, np.uint8)
        for i, r in enumerate(res):
            mv[i, :len(r[0])] = r[0]
        np.savez_compressed(
            os.path.join(OUT, name + ".npz"),
            seed=np.array(seed, np.uint64), game_id0=np.array(g0, np.uint64),
            policy=np.array(policy), n_random=np.array(n_random),
            start_black=u64([s[0] for s in starts]), start_white=u64([s[1] for s in starts]),
            start_turn=np.array([s[2] for s in starts], np.uint8),
            moves=mv, final_black=u64([r[1] for r in res]), final_white=u64([r[2] for r in res]),
            diff=np.array([r[3] for r in res], np.int8), plies=np.array([r[4] for r in res], np.uint8),
            **({} if weights is None else {"weights": np.array(weights, np.int8)}),
            **({} if weights_white is None else {"weights_white": np.array(weights_white, np.int8)}))

    rollouts("rollout_random", SEED, 0, 256, 0, 0)
    rollouts("rollout_random_offset", 12345, (1 << 20) * 3 + 77, 128, 0, 0)
    mid = [(p[0], p[1], p[2]) for p in pos[:128] if p[2] in (Black, White)]
    rollouts("rollout_random_from_mid", 777, 5, len(mid), 0, 0, starts=mid)
    rollouts("rollout_greedy", SEED, 0, 192, 1, 10)
    rollouts("rollout_greedy_from_mid", 99, 1000, 64, 1, 0, starts=mid[:64])

    # ---------------------------------------------------------------- eval policy + linear eval (§8f row 2)
    ns = load_reference_counts(want_ns=True)
    wdef = [list(r) for r in ns["ProgressPositionMovesParameter"]().default_value()]
    wrand = np.random.default_rng(77).integers(-127, 128, (4, 9)).tolist()
    rollouts("rollout_eval", SEED, 0, 128, 2, 10, weights=wdef)
    rollouts("rollout_eval_rand_from_mid", 4242, 77, 64, 2, 0, starts=mid[:64], weights=wrand)
    # a match: the reference's default table as Black against the random table as White
    rollouts("rollout_match", 5150, 9, 128, 2, 6, weights=wdef, weights_white=wrand)
    runner_fixtures(pool)
    boards = [from_bits(p[0], p[1], p[2]) for p in pos[:512]]
    np.savez_compressed(
        os.path.join(OUT, "eval_values.npz"),
        black=u64([p[0] for p in pos[:512]]), white=u64([p[1] for p in pos[:512]]),
        weights_default=np.array(wdef, np.int8), weights_rand=np.array(wrand, np.int8),
        # columns: side 'O', 'X', '-' (any other string: turn_from_string -> Empty)
        counts=np.array([[list(ns["counts"]({"book": b.serialize_board(), "whosturn": b.serialize_turn(), "turn": b.nturn},
                                      sd)) for sd in ("O", "X", "-")] for b in boards], np.uint8),
        eval_default=np.array([[eval_value(b, sd, wdef) for sd in ("O", "X", "-")] for b in boards], np.int32),
        eval_rand=np.array([[eval_value(b, sd, wrand) for sd in ("O", "X", "-")] for b in boards], np.int32))

    # ---------------------------------------------------------------- config-2 generator
    sm = pool.map(sample_midgame, [(SEED, i) for i in range(256)], chunksize=4)
    np.savez_compressed(os.path.join(OUT, "sample_midgame.npz"), seed=np.array(SEED, np.uint64),
                        black=u64([s[0] for s in sm]), white=u64([s[1] for s in sm]),
                        turn=np.array([s[2] for s in sm], np.uint8), nturn=np.array([s[3] for s in sm], np.uint8),
                        move=np.array([s[4] for s in sm], np.uint8))

    # ---------------------------------------------------------------- books (§8f row 1) + features (row 2)
    counts = load_reference_counts()
    z = np.load(os.path.join(OUT, "rollout_random.npz"))
    zm = np.load(os.path.join(OUT, "rollout_random_from_mid.npz"))
    books = []
    for src, g in [(z, i) for i in range(12)] + [(zm, i) for i in range(4)]:
        b = from_bits(int(src["start_black"][g]), int(src["start_white"][g]), int(src["start_turn"][g]))
        lines = [b.serialize_str()]  # FlatFileRecorder.add after Board() (game_runner.py:169-170)
        records = [{"book": b.serialize_board(), "whosturn": b.serialize_turn(), "turn": b.nturn,
                    "end": b.is_game_over()}]
        feats = []
        for code in src["moves"][g]:
            if code == 255:
                break
            assert b.put_s(code_to_str(b, int(code))) >= 0
            lines.append(b.serialize_str())
            records.append({"book": b.serialize_board(), "whosturn": b.serialize_turn(), "turn": b.nturn,
                            "end": b.is_game_over()})
        for rec in records:
            feats.append([list(counts(rec, "O")), list(counts(rec, "X"))])
        books.append({"source": "rollout_random" if src is z else "rollout_random_from_mid", "game": g,
                      "lines": lines, "records": records, "counts": feats})
    json.dump(books, open(os.path.join(OUT, "books.json"), "w"))

    # ---------------------------------------------------------------- TD state map (§8f row 2)
    # ProgressPositionMovesLearn.__update_state_for_a_book / __update_state_map
    # (progress_position_moves_learn.py:37-62) run from the reference module
    # itself (reference_state_map) over the 256 rollout_random games as
    # learn_books hands them over (replearn.py:34-39: records sorted by turn,
    # reversed).
    store = reference_state_map([game_book_learn_order(z, g) for g in range(len(z["plies"]))])
    ks = sorted(store)
    np.savez_compressed(os.path.join(OUT, "td_state.npz"), source=np.array("rollout_random"),
                        games=np.array(len(z["plies"])), hash=np.array(ks), value=np.array([store[k] for k in ks]),
                        draws=np.array(int((z["diff"] == 0).sum())))

    # ---------------------------------------------------------------- RNG known answers
    S = seed_state(SEED)
    r0 = GameRng(game_key(S, 0))
    rng = {"seed": SEED, "seed_state": hex(S),
           "game_keys": [hex(game_key(S, g)) for g in (0, 1, 2, 1 << 20, (1 << 40) + 3)],
           "draws_g0": [r0.draw() for _ in range(8)]}
    json.dump(rng, open(os.path.join(OUT, "rng.json"), "w"), indent=1)
    print("fixtures written to", OUT)


# ----------------------------------------------------------------------------
# §8f row 3: LearnBasePlus.store_batch_stats run from the reference itself
# ----------------------------------------------------------------------------
def load_reference_learn_base():
    """learn_base.py exec'd against the shimmed board module and a stub `slack`
    module (its post_message only records the text: no network).  One in-memory
    substitution, learn_base.py:87's Python 2 print statement -> print(...);
    nothing is written to /root/reference and no source is copied."""
    import types
    src = open("/root/reference/learn_base.py").read()
    a = "print 'Exception occured while processing %d th book' % book_id\n"
    assert src.count(a) == 1, "learn_base.py changed; the shim substitution no longer applies"
    src = src.replace(a, "print('Exception occured while processing %d th book' % book_id)\n")
    mod_board = types.ModuleType("board")
    mod_board.__dict__.update(RB)
    mod_slack = types.ModuleType("slack")
    mod_slack.messages = []
    mod_slack.post_message = mod_slack.messages.append
    saved = {k: sys.modules.get(k) for k in ("board", "slack")}
    sys.modules["board"], sys.modules["slack"] = mod_board, mod_slack
    try:
        ns = {"__name__": "reference_learn_base"}
        exec(compile(src, "reference_learn_base.py", "exec"), ns)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return ns, mod_slack


def load_reference_learner():
    """progress_position_moves_learn.py exec'd as the reference wrote it, with
    its Python 2 print statements (lines 38, 123, 155, 156, 168, 173, 221, 222)
    turned into print(...) calls in memory, and its imports served by:
      * board, parameter, parameter_progress_position_moves_learn, learn_base:
        the reference's own modules, exec'd as above (board.py through its shim);
      * slack: a stub that records the text (no network);
      * pyres, parallel_learner_task, config, replearn: stubs -- they are only
        reached from the Resque fan-out (__fit_parameters, 115-158) and
        configure(), which the state-map update does not touch.
    sklearn and numpy are the real packages.  Nothing is written to
    /root/reference and no source is copied."""
    import re
    import types
    src = open("/root/reference/progress_position_moves_learn.py").read().split("\n")
    print_lines = [i for i, ln in enumerate(src) if re.match(r"\s*print ", ln)]
    assert [i + 1 for i in print_lines] == [38, 123, 155, 156, 168, 173, 221, 222], \
        "progress_position_moves_learn.py changed; the print shim no longer applies"
    for i in print_lines:
        m = re.match(r"(\s*)print (.*?)(\s*#.*)?$", src[i])
        src[i] = "%sprint(%s)%s" % (m.group(1), m.group(2), m.group(3) or "")
    lb_ns, slack = load_reference_learn_base()
    ppml = load_reference_counts(want_ns=True)

    def module(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        return m

    class ResQ:  # pyres: never reached by the state-map update
        def __init__(self, *a, **k):
            raise RuntimeError("pyres stub: the Resque fan-out is out of scope")

    mods = {
        "board": module("board", **RB),
        "slack": slack,
        "learn_base": module("learn_base", **lb_ns),
        "parameter": module("parameter", board_from_a_book=ppml["board_from_a_book"]),
        "parameter_progress_position_moves_learn": module("parameter_progress_position_moves_learn", **ppml),
        "pyres": module("pyres", ResQ=ResQ),
        "parallel_learner_task": module("parallel_learner_task", ParallelLearnerTask=object),
        "config": module("config", redis_hostname_port_from_config=lambda c: None),
        "replearn": module("replearn", get_instance_from_config=None),
    }
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    try:
        ns = {"__name__": "reference_progress_position_moves_learn"}
        exec(compile("\n".join(src), "reference_progress_position_moves_learn.py", "exec"), ns)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return ns, ppml


class RedisLikeStore:
    """The parameter store as RedisParameterStore presents it to the learner
    (redis_parameter_store.py:26-39): values go in as redis-py encodes them
    (repr() of a float, str() of an int) and come back as strings, so float()
    reads back exactly the value set."""

    def __init__(self):
        self.kv = {}

    def exists(self, key):
        return ":".join(key) in self.kv

    def get(self, key):
        return self.kv.get(":".join(key))

    def set(self, key, value):
        self.kv[":".join(key)] = repr(value) if isinstance(value, float) else str(value)
        return True


def reference_state_map(books):
    """{hash: value} after ProgressPositionMovesLearn.__update_state_for_a_book
    (progress_position_moves_learn.py:37-48) -> __update_state_map (50-62), the
    reference's own code, over `books` in order (learn_and_update_batch, 88-91).
    The learner's print of each terminal record (line 38) is discarded."""
    import contextlib
    import io
    ns, ppml = load_reference_learner()
    store = RedisLikeStore()

    class Learner(ns["ProgressPositionMovesLearn"]):
        def _param_store(self):
            return store

    lrn = Learner()
    lrn.parameter = ppml["ProgressPositionMovesParameter"]()  # what configure() instantiates
    update = lrn._ProgressPositionMovesLearn__update_state_for_a_book
    with contextlib.redirect_stdout(io.StringIO()):
        for i, book in enumerate(books):
            update(i, book)
    prefix = "param:state:"
    assert all(k.startswith(prefix) for k in store.kv)
    return {k[len(prefix):]: float(v) for k, v in store.kv.items()}


def game_book_learn_order(z, g):
    """Game g of a rollout fixture as the recorder writes it (the record after
    Board() and after every put_s, game_runner.py:169-184) and learn_books hands
    it to the learner: sorted by turn, reversed (replearn.py:34-39)."""
    ib, iw = to_bits(Board())
    b = from_bits(ib, iw, Black)
    recs = [{"book": b.serialize_board(), "whosturn": b.serialize_turn(), "turn": b.nturn, "end": b.is_game_over()}]
    for code in z["moves"][g]:
        if code == 255:
            break
        assert b.put_s(code_to_str(b, int(code))) >= 0
        recs.append({"book": b.serialize_board(), "whosturn": b.serialize_turn(), "turn": b.nturn,
                     "end": b.is_game_over()})
    return list(reversed(sorted(recs, key=lambda x: int(x["turn"]))))


def replay_terminal(sb, sw, st, moves):
    """The terminal record a game's recorder writes (game_recorder.py:107-114):
    the board after the recorded move codes, driven through board.py's put_s."""
    b = from_bits(int(sb), int(sw), int(st))
    for c in moves:
        if c == 0xFF:
            break
        b.put_s(code_to_str(b, int(c)))
    return {"book": b.serialize_board(), "whosturn": b.serialize_turn(), "turn": b.nturn, "end": True}


def batch_stats_fixtures():
    """batch_stats.json: books -> the (key, payload) LearnBasePlus.store_batch_stats
    (learn_base.py:58-110) hands its parameter store's hmset, run from the
    reference.  The payload's params_used joins a set: its order is the set's
    iteration order, which Python 3 randomises per process for strings, so the
    generator runs under PYTHONHASHSEED=0 and records that."""
    import fnmatch
    import subprocess
    if os.environ.get("PYTHONHASHSEED") != "0":
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--only", "batch_stats", "--out", OUT],
                              env=dict(os.environ, PYTHONHASHSEED="0"))
        return
    ns, slack = load_reference_learn_base()

    class Store:  # the ParameterStore calls store_batch_stats and __show_stats make
        def __init__(self):
            self.calls, self.h = [], {}

        def configure(self, conf):
            pass

        def hmset(self, key, mapping):
            self.calls.append((list(key), dict(mapping)))
            self.h[":".join(key)] = dict(mapping)

        def keys(self, pattern):
            return [k for k in self.h if fnmatch.fnmatch(k, ":".join(pattern))]

        def hgetall(self, k):
            return self.h[k]

    class RefLearn(ns["LearnBasePlus"]):
        def __init__(self):
            super().__init__()
            self.store = Store()

        def name(self):
            return "gpu"

        def _param_store(self):
            return self.store

    def run(books):
        lrn = RefLearn()
        lrn.store_batch_stats([(i, [dict(r) for r in recs] if isinstance(recs, list) else recs,
                                dict(m) if isinstance(m, dict) else m) for i, recs, m in books])
        assert len(lrn.store.calls) == 1
        return lrn.store.calls[0]

    cases = []

    def case(name, books, note=""):
        key, payload = run(books)
        cases.append({"name": name, "note": note, "books": [list(b) for b in books], "key": key, "payload": payload})

    def fixture_books(src, meta, id0=None, params=None):
        z = np.load(os.path.join(OUT, src + ".npz"), allow_pickle=False)
        g0 = int(z["game_id0"]) if id0 is None else id0
        books = []
        for i in range(len(z["final_black"])):
            term = replay_terminal(z["start_black"][i], z["start_white"][i], z["start_turn"][i], z["moves"][i])
            m = dict(meta)
            if params:
                m["hamletparam"] = params[i % len(params)]
            books.append((g0 + i, [term, {"book": "", "whosturn": "O", "turn": 0, "end": False}], m))
            # the replayed terminal board is the fixture's final board
            b = Board()
            b.deserialize(term["book"], term["whosturn"], term["turn"])
            fb, fw = to_bits(b)
            assert (fb, fw) == (int(z["final_black"][i]), int(z["final_white"][i])), (src, i)
        return books

    meta = {"proc_a": "Edax", "proc_b": "Hamlet", "hamletparam": "p0"}
    for src in ("rollout_random", "rollout_greedy", "rollout_random_from_mid", "rollout_match"):
        case(src, fixture_books(src, meta), "terminal records replayed through board.py from the fixture's moves")
    case("multi_param", fixture_books("rollout_random_offset", meta, params=["pA", "pB", "pC"]),
         "three hamletparam values: params_used is ' / '.join(set) in the generator's set order (PYTHONHASHSEED=0)")
    # line 77: a Black win, then two draws; White's discs are compared with the
    # running count of Black wins, so both draws count as White wins
    full, half = (1 << 64) - 1, (1 << 32) - 1

    def rec(bl, wh, turn="O"):
        return {"book": from_bits(bl, wh, Black).serialize_board(), "whosturn": turn, "turn": 60, "end": True}

    case("line77", [(0, [rec(full ^ 1, 1)], meta), (1, [rec(half, full ^ half)], meta),
                    (2, [rec(0xFF, 0xFF00)], meta)], "Black win then two draws")
    # malformed books: learn_base.py:66-88's try (tests/test_stats.py shapes)
    rng = np.random.default_rng(0)
    bl = rng.integers(0, 2**63, 12, dtype=np.int64).astype(np.uint64) << np.uint64(1)
    wh = rng.integers(0, 2**63, 12, dtype=np.int64).astype(np.uint64) & ~bl
    books = [(100 + i, [rec(int(bl[i]), int(wh[i]))], dict(meta)) for i in range(12)]
    books[1] = (101, [], dict(meta))                                      # empty book: IndexError at book[0]
    books[2][1][0]["book"] += "O"                                          # 65 cells: IndexError in deserialize
    books[3][1][0]["book"] = "XXXXOOOO"                                    # short: over Board()'s opening
    del books[4][1][0]["whosturn"]                                         # KeyError before counting
    books[5] = (105, books[5][1], {"proc_a": "C"})                        # counted; names stop at proc_b
    books[6] = (106, books[6][1], None)                                   # counted; meta unreadable
    books[7] = (107, books[7][1], {"proc_a": "D", "proc_b": "E", "hamletparam": "p1"})
    books[8][1][0]["book"] = "".join(rng.choice(list("OX-?o "), 64))      # other characters -> Empty
    case("malformed", books, "learn_base.py:85-88: a book that raises stops where it raised, "
                             "and still counts in len(books)")
    out = {"source": "/root/reference/learn_base.py:58-110 exec'd by gen_golden.py (print shim at :87, "
                     "stub slack, dict parameter store)",
           "pythonhashseed": os.environ.get("PYTHONHASHSEED"), "cases": cases}
    json.dump(out, open(os.path.join(OUT, "batch_stats.json"), "w"))
    print("batch_stats.json:", len(cases), "cases;", len(slack.messages), "slack messages captured")


def td_records_fixtures():
    """The learner's state-map update over books that are not clean GameRunner
    games (books read from any store: td.StateMap.update_from_records).
    __update_state_for_a_book / __update_state_map
    (progress_position_moves_learn.py:37-62) over each book in the given order,
    run from the reference module itself (reference_state_map).  Books are built from rollout_random.npz games replayed through
    board.py, then altered: records dropped (gaps in turn), repeated, shuffled
    after the terminal, turns as strings, board strings cut short (the rest of
    the squares stay the opening's) or holding other characters ('o', 'x',
    '.', ...: Empty), and boards of random characters."""
    z = np.load(os.path.join(OUT, "rollout_random.npz"))
    rnd = random.Random(20261017)
    books, kinds = [], []
    for g in range(40):
        book = game_book_learn_order(z, g)
        kind = ["clean", "gaps", "repeats", "shuffled", "str_turns", "short", "chars", "random_boards"][g % 8]
        if kind == "gaps":
            book = [book[0]] + [r for r in book[1:] if rnd.random() < 0.6]
        elif kind == "repeats":
            book = [book[0]] + [r for r in book[1:] for _ in range(1 + (rnd.random() < 0.3))]
        elif kind == "shuffled":
            rest = book[1:]
            rnd.shuffle(rest)
            book = [book[0]] + rest
        elif kind == "str_turns":
            book = [dict(r, turn=str(r["turn"])) for r in book]
        elif kind == "short":
            book = [dict(r, book=r["book"][:rnd.randrange(0, 65)]) for r in book]
        elif kind == "chars":
            book = [dict(r, book="".join(c if rnd.random() < 0.8 else rnd.choice("ox.* #0") for c in r["book"]))
                    for r in book]
        elif kind == "random_boards":
            book = [dict(r, book="".join(rnd.choice("OX-OX-ox.") for _ in range(64))) for r in book]
        books.append(book)
        kinds.append(kind)
    # learn_and_update_batch (88-91) -> __update_state_for_a_book (37-48), run from the reference
    store = reference_state_map(books)
    ks = sorted(store)
    out = {"source": "progress_position_moves_learn.py:37-62 exec'd from the reference (reference_state_map) over "
                     "rollout_random.npz games replayed through board.py and altered",
           "kinds": kinds, "books": books, "hash": ks, "value": [store[k] for k in ks]}
    json.dump(out, open(os.path.join(OUT, "td_records.json"), "w"))
    print("td_records.json:", len(books), "books,", sum(map(len, books)), "records,", len(ks), "keys")


if __name__ == "__main__":
    if "--out" in sys.argv:  # another directory (tests/test_golden_regen.py regenerates into a temp dir)
        OUT = os.path.abspath(sys.argv[sys.argv.index("--out") + 1])
        os.makedirs(OUT, exist_ok=True)
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    if only == "batch_stats":
        batch_stats_fixtures()
    elif only == "td_records":
        td_records_fixtures()
    elif only == "runner":
        runner_fixtures(mp.Pool(8))
        print("runner fixtures written to", OUT)
    else:
        # every fixture: main() writes the rollouts the last two read
        main()
        batch_stats_fixtures()
        td_records_fixtures()
