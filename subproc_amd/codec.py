"""Host-side text codecs of the reference (not on the compute path).

* Edax-protocol move strings <-> integer move codes (0..63 = x + 8*y, 64 = pass):
  board.py:176-209 (coord_from_handstr / handstr_from_coord / put_s) and the
  engine reply formats of game_runner.py:27, 51.
* Book text <-> bitboards: board.py:211-262 (serialize_* / deserialize), the
  record format of game_recorder.py:62-76, 107-114, 197-205.
  Book text uses 'O' = Black, 'X' = White, '-' = empty, row-major a1..h8.
"""
import re

import numpy as np

EMPTY, BLACK, WHITE = 0, 1, 2
PASS = 64
INVALID = 255  # a code the C-ABI answers with ret = -1 (unparsable move)

_HAND_RE = re.compile(r"[WB]*([a-zA-Z])([0-9])")  # board.py:177
_ENGINE_GO_RE = re.compile(r">(.+) plays [WB]?([a-zA-Z][0-9]|PS)")  # game_runner.py:27
_ENGINE_PLAY_RE = re.compile(r"(.+) play ([a-zA-Z][0-9]|PS|ps)")  # game_runner.py:51


def coord_from_handstr(handstr):
    """board.py:176-185: first ``[WB]*<letter><digit>`` match -> (x, y), else (-1, -1)."""
    b = _HAND_RE.findall(handstr)
    if b:
        col, row = b[0][0].lower(), b[0][1]
        return ord(col) - ord("a"), ord(row) - ord("1")
    return -1, -1


def handstr_from_coord(x, y):
    """board.py:187-190."""
    return chr(ord("a") + x) + chr(ord("1") + y)


def move_code(stri):
    """Edax move string -> integer code, with board.py:192-209 semantics:

    'PS' / 'ps' -> 64; an unparsable string or a negative coordinate -> 255
    (put_s answers -1); an on-board square -> x + 8*y.  A coordinate past the
    edge ('a9', 'i1') raises IndexError exactly as board.py:162 does.
    """
    if stri == "PS" or stri == "ps":
        return PASS
    x, y = coord_from_handstr(stri)
    if x >= 0 and y >= 0:
        if x >= 8 or y >= 8:
            raise IndexError("list index out of range")
        return x + 8 * y
    return INVALID


def move_str(code):
    """Integer code -> Edax move string ('ps' for a pass; game_runner lowercases, 152)."""
    if code == PASS:
        return "ps"
    if not 0 <= code < 64:
        raise ValueError(f"not a move code: {code}")
    return handstr_from_coord(code % 8, code // 8)


def parse_engine_go(output):
    """Engine reply to 'go' (game_runner.py:19-33): returns (name, move code)."""
    b = _ENGINE_GO_RE.findall(output.rstrip())
    return b[0][0], move_code(b[0][1].lower())


def parse_engine_play(output):
    """Engine echo of a played move (game_runner.py:41-54): returns the move code."""
    a = _ENGINE_PLAY_RE.findall(output.rstrip())
    return move_code(a[0][1].lower())


# ---------------------------------------------------------------------------
# book text
# ---------------------------------------------------------------------------
def string_from_turn(turn):
    """board.py:237-243."""
    return "O" if turn == BLACK else "X" if turn == WHITE else "-"


def turn_from_string(s):
    """board.py:245-251."""
    return BLACK if s == "O" else WHITE if s == "X" else EMPTY


def serialize_board(black, white):
    """board.py:223-232 for one (black, white) bitboard pair."""
    return "".join("O" if black >> sq & 1 else "X" if white >> sq & 1 else "-" for sq in range(64))


def serialize_str(black, white, turn, append_turn=True):
    """board.py:214-221."""
    s = serialize_board(black, white)
    return s + " " + string_from_turn(turn) if append_turn else s


def deserialize_board(board_str, black=0, white=0):
    """board.py:253-258: cell i of the string sets square (i % 8, i // 8); a
    string shorter than 64 leaves the remaining squares as they were, a longer
    one raises IndexError (row 8 does not exist)."""
    for i, s in enumerate(board_str):
        if i >= 64:
            raise IndexError("list index out of range")
        bit = 1 << i
        black &= ~bit
        white &= ~bit
        c = turn_from_string(s)
        if c == BLACK:
            black |= bit
        elif c == WHITE:
            white |= bit
    return black, white


# batched (numpy) versions for book emission / ingestion
_LUT = np.frombuffer(b"-OX", dtype=np.uint8)


def serialize_boards(boards):
    """(n, 2) uint64 [black, white] -> list of 64-char book strings (vectorised)."""
    b = np.ascontiguousarray(boards, dtype=np.uint64)
    sq = np.arange(64, dtype=np.uint64)
    bl = ((b[:, :1] >> sq) & np.uint64(1)).astype(np.uint8)
    wh = ((b[:, 1:] >> sq) & np.uint64(1)).astype(np.uint8)
    chars = _LUT[bl + 2 * wh]
    return [row.tobytes().decode() for row in chars]


def deserialize_boards(strings):
    """list of 64-char book strings -> (n, 2) uint64 (vectorised, full 64-char strings only)."""
    a = np.frombuffer("".join(strings).encode(), dtype=np.uint8).reshape(len(strings), 64)
    w = np.uint64(1) << np.arange(64, dtype=np.uint64)
    black = ((a == ord("O")).astype(np.uint64) * w).sum(axis=1, dtype=np.uint64)
    white = ((a == ord("X")).astype(np.uint64) * w).sum(axis=1, dtype=np.uint64)
    return np.stack([black, white], axis=1)
