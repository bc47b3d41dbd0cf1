"""Host-side codecs (Edax move strings, book text) against board.py fixtures; CPU only."""
import numpy as np
import pytest

from golden_io import load_json, load_npz
from subproc_amd import codec
from subproc_amd import board as gboard


def test_move_strings_match_put_s_parse():
    op = load_json("opening.json")
    for rec in op["strings"]:
        code = codec.move_code(rec["s"])
        if rec["ret"] == 0:
            assert code == codec.PASS, rec["s"]
        elif rec["ret"] == -1 and code != codec.INVALID:
            assert 0 <= code < 64  # parsed but illegal on the board: the kernel answers -1
        else:
            assert 0 <= code < 64 or code == codec.INVALID
    for m in op["moves"]:
        assert codec.move_code(m["move"]) == m["sq"]
        assert codec.move_str(m["sq"]) == m["move"]
    for rec in op["index_error"]:
        if rec["raises"]:
            with pytest.raises(IndexError):
                codec.move_code(rec["s"])


def test_coord_from_handstr_cases():
    assert codec.coord_from_handstr("d3") == (3, 2)
    assert codec.coord_from_handstr("BWf5") == (5, 4)
    assert codec.coord_from_handstr("xyz") == (-1, -1)
    assert codec.coord_from_handstr("a0") == (0, -1)
    assert codec.move_code("a0") == codec.INVALID
    assert codec.move_code("Ps") == codec.INVALID
    assert codec.handstr_from_coord(7, 7) == "h8"


def test_engine_reply_parsing():
    assert codec.parse_engine_go(">Edax plays WD3") == ("Edax", 19)
    assert codec.parse_engine_go(">Hamlet plays PS") == ("Hamlet", 64)
    assert codec.parse_engine_play("Edax play c4") == 26


def test_serialize_matches_fixture():
    op = load_json("opening.json")
    b = gboard.Board()
    assert b.serialize_str() == op["serialize_str"]
    assert b.serialize_board() == op["serialize_board"]
    for e in load_json("edges.json"):
        s = codec.serialize_str(int(e["black"], 16), int(e["white"], 16), e["turn"])
        assert s == e["serialize_str"], e["name"]


def test_deserialize_roundtrip_and_batch():
    z = load_npz("midgame_step.npz")
    boards = np.stack([z["black"], z["white"]], 1)[:300]
    strs = codec.serialize_boards(boards)
    for (bl, wh), s in zip(boards[:50], strs[:50]):
        assert s == codec.serialize_board(int(bl), int(wh))
        assert codec.deserialize_board(s) == (int(bl), int(wh))
    np.testing.assert_array_equal(codec.deserialize_boards(strs), boards)


def test_board_facade_host_state():
    b = gboard.Board()
    assert b.turn == gboard.Black and b.nturn == 0
    assert b.get(3, 3) == gboard.White and b.get(4, 3) == gboard.Black
    b.deserialize("-" * 64, "X", 7)
    assert b.bitboards() == (0, 0) and b.turn == gboard.White and b.nturn == 7
    b.set(gboard.Black, 0, 0)
    assert b.board[0][0] == gboard.Black
    assert gboard.clone_board(b.board) == b.board
    assert gboard.is_within_board(7, 7) and not gboard.is_within_board(8, 0)
    assert b.mask_count(gboard.Black, 1) == 1
    with pytest.raises(IndexError):
        b.deserialize("-" * 65, "O", 0)
