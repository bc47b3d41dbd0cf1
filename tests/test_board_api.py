"""board.py's answers beyond Black/White play, bit-exact:

* the side to move Empty (deserialize with '-') or a value no square holds,
  through put_s / puttables (board.py:46-58, 155-159, 192-209);
* put / is_puttable_at / get / set at Python-wrapped coordinates -8..-1 and
  hands_for_direc from any origin along any direction (board.py:60-64,
  124-174);
* the live ``board`` list, cells holding other values, deserialize edge cases.

Fixtures: tests/golden/board_api.{npz,json} and side_steps.npz, made by
gen_golden.py from the real board.py.  The oracle and the host build of the
C-ABI are checked here on CPU; the facade runs on both backends
(tests/facade_backends.py: libothello_cpu.so here, the HIP library under -m gpu).
"""
import ctypes

import numpy as np
import pytest

import oracle
from facade_backends import facade  # noqa: F401  (pytest fixture)
from golden_io import load_json, load_npz

P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
API = load_npz("board_api.npz")
SIDE = load_npz("side_steps.npz")
PIECES = [int(p) for p in API["pieces"]]
XY = [int(v) for v in API["xy"]]


def _cells(b):
    return [[c if isinstance(c, int) else str(c) for c in row] for row in b.board]


# --------------------------------------------------------------------------- oracle / host C-ABI
def test_oracle_side_to_move_empty_and_other():
    b = np.stack([SIDE["black"], SIDE["white"]], 1)
    n = len(b)
    np.testing.assert_array_equal(oracle.legal(b, SIDE["turn"]), SIDE["legal"])
    for code in range(65):
        r = oracle.step(b, SIDE["turn"], np.full(n, code, np.uint8), nturn=np.full(n, 7, np.uint8))
        np.testing.assert_array_equal(r["ret"], SIDE["ret"][:, code])
        np.testing.assert_array_equal(r["boards"][:, 0], SIDE["next_black"][:, code])
        np.testing.assert_array_equal(r["boards"][:, 1], SIDE["next_white"][:, code])
        np.testing.assert_array_equal(r["turn"], SIDE["next_turn"][:, code])
        np.testing.assert_array_equal(r["nturn"], SIDE["next_nturn"][:, code])
        np.testing.assert_array_equal(r["legal_next"], SIDE["next_legal"][:, code])


def _hands_items():
    """Every (board, piece, direction, y, x) of the fixture as flat columns."""
    nb, npc, nd, ny, nx = API["hands"].shape
    ib, ip, idr, iy, ix = np.meshgrid(np.arange(nb), np.arange(npc), np.arange(nd), np.arange(ny), np.arange(nx),
                                      indexing="ij")
    ib, ip, idr, iy, ix = (a.reshape(-1) for a in (ib, ip, idr, iy, ix))
    sx = API["scan_xy"]
    return dict(board=ib, piece=API["pieces"][ip], dx=API["scan_direcs"][idr, 0], dy=API["scan_direcs"][idr, 1],
                x=sx[ix], y=sx[iy], want=API["hands"].reshape(-1))


def own_hostile(black, white, piece):
    """Squares holding `piece` / hostile(piece) (board.py:155-159) on a Black/White board."""
    occ = black | white
    own = np.where(piece == 1, black, np.where(piece == 2, white, np.where(piece == 0, ~occ, np.uint64(0))))
    return own.astype(np.uint64), np.where(piece == 1, white, black).astype(np.uint64)


def test_oracle_hands_any_origin_any_direction():
    it = _hands_items()
    b = np.stack([API["black"][it["board"]], API["white"][it["board"]]], 1)
    got = oracle.hands(b, it["piece"], it["x"], it["y"], it["dx"], it["dy"])
    np.testing.assert_array_equal(got, it["want"])


def test_cpu_abi_hands_own_hostile_form():
    it = _hands_items()
    own, hos = own_hostile(API["black"][it["board"]], API["white"][it["board"]], it["piece"])
    n = len(own)
    out = np.zeros(n, np.uint8)
    cols = [np.ascontiguousarray(it[k], np.int64) for k in ("x", "y", "dx", "dy")]
    assert oracle.cpu_abi().oth_hands(P(own), P(hos), *[P(c) for c in cols], P(out), n, None) == 0
    np.testing.assert_array_equal(out, it["want"])


# --------------------------------------------------------------------------- the facade (both backends)
def test_facade_put_and_is_puttable_at_wrapped_coordinates(facade):  # noqa: F811
    for i in range(len(API["black"])):
        bl, wh = int(API["black"][i]), int(API["white"][i])
        for pi, piece in enumerate(PIECES):
            b0 = facade.Board()
            b0._set_bits(bl, wh)
            for iy, y in enumerate(XY):
                for ix, x in enumerate(XY):
                    assert b0.is_puttable_at(piece, x, y) == bool(API["puttable"][i, pi, iy, ix]), (i, piece, x, y)
                    b = facade.Board()
                    b._set_bits(bl, wh)
                    r = b.put(piece, x, y)
                    assert r == int(API["put_ret"][i, pi, iy, ix]), (i, piece, x, y)
                    assert b.bitboards() == (int(API["put_black"][i, pi, iy, ix]),
                                             int(API["put_white"][i, pi, iy, ix])), (i, piece, x, y)
            m = sum(1 << (x + 8 * y) for x, y in b0.puttables(piece))
            assert m == int(API["legal"][i, pi]), (i, piece)
            assert b0.n_puttable_for(piece) == bin(m).count("1")


def test_facade_out_of_range_index_raises(facade):  # noqa: F811
    b = facade.Board()
    for x, y in ((8, 0), (0, 8), (-9, 0), (0, -9)):
        with pytest.raises(IndexError):
            b.put(1, x, y)
        with pytest.raises(IndexError):
            b.is_puttable_at(1, x, y)
        with pytest.raises(IndexError):
            b.get(x, y)
        with pytest.raises(IndexError):
            b.set(1, x, y)


def test_facade_hands_for_direc_any_origin(facade):  # noqa: F811
    sx = [int(v) for v in API["scan_xy"]]
    for i in (0, 24, 26, 28):  # a mid-game board, row 1 White, the a1-h8 diagonal, the put-order board
        b = facade.Board()
        b._set_bits(int(API["black"][i]), int(API["white"][i]))
        for pi, piece in enumerate(PIECES):
            for di, (dx, dy) in enumerate(API["scan_direcs"].tolist()):
                for iy, y in enumerate(sx):
                    for ix, x in enumerate(sx):
                        k = int(API["hands"][i, pi, di, iy, ix])
                        want = [(piece, x + j * dx, y + j * dy) for j in range(1, k + 1)]
                        assert b.hands_for_direc((dx, dy), piece, x, y) == want, (i, piece, dx, dy, x, y)


def test_facade_side_to_move_empty_and_other(facade):  # noqa: F811
    for c in list(range(0, 32)) + list(range(256, 288)):
        turn = int(SIDE["turn"][c])
        for code in range(65):
            b = facade.Board()
            b._set_bits(int(SIDE["black"][c]), int(SIDE["white"][c]))
            if turn == 0:
                b.deserialize(b.serialize_board(), "-", 7)
            else:
                b.turn, b.nturn = turn, 7
            if code == 0:
                m = sum(1 << (x + 8 * y) for x, y in b.puttables(b.turn))
                assert m == int(SIDE["legal"][c])
            s = "ps" if code == 64 else b.handstr_from_coord(code % 8, code // 8)
            assert b.put_s(s) == int(SIDE["ret"][c, code]), (c, code)
            assert b.bitboards() == (int(SIDE["next_black"][c, code]), int(SIDE["next_white"][c, code]))
            assert b.turn == int(SIDE["next_turn"][c, code]) and b.nturn == int(SIDE["next_nturn"][c, code])
            m = sum(1 << (x + 8 * y) for x, y in b.puttables(b.turn))
            assert m == int(SIDE["next_legal"][c, code]), (c, code)


def _apply(b, ops):
    for op in ops:
        if op[0] == "board":
            b.board[op[1]][op[2]] = op[3]
        else:
            b.set(op[1], op[2], op[3])


def test_facade_live_board_and_other_values(facade):  # noqa: F811
    fx = load_json("board_api.json")
    for rec in fx["boards"]:
        b = facade.Board()
        _apply(b, rec["ops"])
        name = rec["name"]
        assert _cells(b) == rec["cells"], name
        assert (b.n_black(), b.n_white(), b.n_empty()) == (rec["n_black"], rec["n_white"], rec["n_empty"]), name
        assert b.is_game_over() == rec["is_game_over"], name
        assert b.serialize_str() == rec["serialize_str"] and str(b) == rec["str"], name
        for p, want in rec["puttables"].items():
            assert [list(t) for t in b.puttables(int(p))] == want, (name, p)
        for p, want in rec["mask_count"].items():
            assert b.mask_count(int(p), 0x00FFFF0000FFFF00) == want, (name, p)
        got = [b.get(x, y) for (x, y) in ((-1, -1), (3, 2), (-5, -6), (2, 3))]
        assert [g if isinstance(g, int) else str(g) for g in got] == rec["get"], name
        for s in rec["put_s"]:
            c = facade.Board()
            _apply(c, rec["ops"])
            code = s["code"]
            mv = "ps" if code == 64 else c.handstr_from_coord(code % 8, code // 8)
            assert c.put_s(mv) == s["ret"], (name, code)
            assert c.turn == s["turn"] and _cells(c) == s["cells"], (name, code)
        for s in rec["put"]:
            c = facade.Board()
            _apply(c, rec["ops"])
            assert c.put(s["piece"], s["x"], s["y"]) == s["ret"], (name, s)
            assert _cells(c) == s["cells"], (name, s)


def test_facade_board_view_is_a_list_of_lists(facade):  # noqa: F811
    b = facade.Board()
    rows = [row[:] for row in b.board]
    assert rows[3][3] == 2 and rows[3][4] == 1 and len(b.board) == 8 and len(b.board[0]) == 8
    assert b.board == rows and b.board[3] == rows[3]
    b.board[0] = [1] * 8
    assert b.get(5, 0) == 1 and b.n_black() == 10
    c = facade.Board()
    c.board = b.board  # whole-board assignment (a clone, as clone_board callers do)
    assert c.bitboards() == b.bitboards()
    assert facade.clone_board(b.board) == rows[:0] + [[1] * 8] + rows[1:]
    with pytest.raises(ValueError):
        b.board[2] = [0] * 7


def test_facade_deserialize_edge_cases(facade):  # noqa: F811
    for rec in load_json("board_api.json")["deserialize"]:
        b = facade.Board()
        if rec["raises"]:
            with pytest.raises(IndexError):
                b.deserialize(rec["board"], rec["turn_str"], 3)
        else:
            b.deserialize(rec["board"], rec["turn_str"], 3)
        assert _cells(b) == rec["cells"] and b.turn == rec["turn"] and b.nturn == rec["nturn"], rec["board"][:8]
