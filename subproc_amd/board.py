"""Drop-in ``board`` module: the reference ``Board`` class API (board.py:20-276)
served by the MI355X kernels.

Callers of the reference (game_runner.py:3, learn_base.py:1, parameter.py:2)
run unchanged with ``sys.modules['board'] = subproc_amd.board``.
Same method names, argument order, colour values (Empty 0, Black 1, White 2),
return codes and Edax move strings.

The rules themselves — legal moves, flips, pass/terminal, disc counts — are
computed by the HIP library (one batch-of-one launch per call, through
subproc_amd.ops); this class keeps only the two bitboards, the side to move and
the ply counter on the host, plus the text codecs.  For throughput use the
batched :class:`subproc_amd.env.VecEnv` / :mod:`subproc_amd.ops` instead.

Documented deviations:
  * ``put``/``hands_for_direc``/``is_puttable_at`` with an off-board (x, y),
    including negative ones that Python list indexing would wrap, raise IndexError;
  * a side to move other than Black/White (only reachable via deserialize of a
    turn string other than 'O'/'X') makes ``put_s`` return -1 for every move.
"""
import numpy as np

from . import codec

COLORS = (Empty, Black, White) = range(0, 3)  # board.py:3-7

DIRECS = (LU, U, RU, L, R, LD, D, RD) = [  # board.py:9-17
    (-1, -1), (0, -1), (1, -1),
    (-1, 0), (1, 0),
    (-1, 1), (0, 1), (1, 1),
]

_OPEN_BLACK = 0x0000000810000000  # board.py:25  e4, d5
_OPEN_WHITE = 0x0000001008000000  # board.py:24  d4, e5


def _i64(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def _u64(x):
    return x & ((1 << 64) - 1)


class _Device:
    """Resident batch-of-one device buffers shared by all Board instances."""

    def __init__(self):
        import torch

        from . import _lib, ops

        _lib.load()
        if not torch.cuda.is_available():
            raise _lib.OthelloLibraryError("subproc_amd.board needs a ROCm GPU: there is no CPU path")
        self.torch, self.ops = torch, ops
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.boards = torch.empty((1, 2), dtype=torch.int64, device=self.dev)
        self.turn = torch.empty(1, dtype=torch.uint8, device=self.dev)
        self.move = torch.empty(1, dtype=torch.uint8, device=self.dev)
        self.host = torch.empty(4, dtype=torch.int64).pin_memory()

    def _load(self, black, white, turn=None, move=None):
        h = self.host
        h[0], h[1] = _i64(black), _i64(white)
        h[2] = 0 if turn is None else turn
        h[3] = 0 if move is None else move
        self.boards.view(-1).copy_(h[:2], non_blocking=True)
        self.turn.copy_(h[2:3], non_blocking=True)
        self.move.copy_(h[3:4], non_blocking=True)

    def legal(self, black, white, piece):
        self._load(black, white, piece)
        return _u64(int(self.ops.legal(self.boards, self.turn).item()))

    def result(self, black, white):
        self._load(black, white)
        r = self.ops.result(self.boards)
        t = self.torch.stack([r.n_black.long(), r.n_white.long(), r.terminal.long()]).view(-1).tolist()
        return t[0], t[1], bool(t[2])

    def step(self, black, white, turn, code):
        self._load(black, white, turn, code)
        r = self.ops.step(self.boards, self.turn, self.move, want_legal=False)
        v = self.torch.cat([r.boards.view(-1), r.flips, r.ret.long()]).tolist()
        return _u64(v[0]), _u64(v[1]), _u64(v[2]), int(v[3])


_DEV = None


def _device():
    global _DEV
    if _DEV is None:
        _DEV = _Device()
    return _DEV


def _check_xy(x, y):
    if not (0 <= x < 8 and 0 <= y < 8):
        raise IndexError("list index out of range")


class Board:
    """board.py:20 — one game; hot-path methods run on the GPU."""

    def __init__(self):  # board.py:22-27
        self._black = _OPEN_BLACK
        self._white = _OPEN_WHITE
        self.turn = Black
        self.nturn = 0
        self._cache = {}

    # ---------------------------------------------------------------- state
    @property
    def board(self):
        """list-of-lists view ``board[y][x]`` (a fresh copy, board.py:23)."""
        return [[self.get(x, y) for x in range(8)] for y in range(8)]

    @board.setter
    def board(self, rows):
        bl = wh = 0
        for y in range(8):
            for x in range(8):
                c = rows[y][x]
                if c == Black:
                    bl |= 1 << (x + 8 * y)
                elif c == White:
                    wh |= 1 << (x + 8 * y)
        self._set_bits(bl, wh)

    def _set_bits(self, black, white):
        self._black, self._white = black, white
        self._cache.clear()

    def bitboards(self):
        """(black, white) uint64 bitboards, sq = x + 8*y."""
        return self._black, self._white

    def set(self, piece, x, y):  # board.py:60-61
        _check_xy(x, y)
        bit = 1 << (x + 8 * y)
        bl, wh = self._black & ~bit, self._white & ~bit
        if piece == Black:
            bl |= bit
        elif piece == White:
            wh |= bit
        self._set_bits(bl, wh)

    def get(self, x, y):  # board.py:63-64
        _check_xy(x, y)
        sq = x + 8 * y
        return Black if self._black >> sq & 1 else White if self._white >> sq & 1 else Empty

    # ---------------------------------------------------------------- GPU-backed rules
    def _result(self):
        k = ("result", self._black, self._white)
        if k not in self._cache:
            self._cache[k] = _device().result(self._black, self._white)
        return self._cache[k]

    def _legal(self, piece):
        if piece not in (Black, White):
            return 0
        k = ("legal", self._black, self._white, piece)
        if k not in self._cache:
            self._cache[k] = _device().legal(self._black, self._white, piece)
        return self._cache[k]

    def count_over_board(self, fun):  # board.py:29-35
        return sum(1 for y in range(8) for x in range(8) if fun(self.get(x, y)))

    def n_black(self):  # board.py:37-38
        return self._result()[0]

    def n_white(self):  # board.py:40-41
        return self._result()[1]

    def n_empty(self):  # board.py:43-44
        nb, nw, _ = self._result()
        return 64 - nb - nw

    def puttables(self, piece):  # board.py:46-52 (row-major == LSB-first)
        m = self._legal(piece)
        out = []
        while m:
            sq = (m & -m).bit_length() - 1
            out.append((sq % 8, sq // 8))
            m &= m - 1
        return out

    def n_puttable_for(self, piece):  # board.py:54-55
        return bin(self._legal(piece)).count("1")

    def is_game_over(self):  # board.py:57-58
        return self._result()[2]

    def is_puttable_at(self, piece, x, y):  # board.py:141-149
        _check_xy(x, y)
        return bool(self._legal(piece) >> (x + 8 * y) & 1)

    def hands_for_direc(self, direc, piece, x, y):  # board.py:124-139
        """Discs captured along one ray from (x, y), as [(piece, nx, ny), ...].
        The ray scan ignores what stands on (x, y) itself, so the flip mask is
        taken from the GPU step on the board with the origin square cleared."""
        _check_xy(x, y)
        if piece not in (Black, White):
            raise ValueError("piece must be Black or White")
        bit = 1 << (x + 8 * y)
        _, _, fl, _ = _device().step(self._black & ~bit, self._white & ~bit, piece, x + 8 * y)
        dx, dy = direc
        ret = []
        for i in range(1, 9):
            nx, ny = x + i * dx, y + i * dy
            if not (0 <= nx < 8 and 0 <= ny < 8) or not fl >> (nx + 8 * ny) & 1:
                break
            ret.append((piece, nx, ny))
        return ret

    def set_hands(self, hands):  # board.py:151-153
        for (piece, x, y) in hands:
            self.set(piece, x, y)

    def hostile(self, piece):  # board.py:155-159
        return White if piece == Black else Black

    def put(self, piece, x, y):  # board.py:161-174 — flips, no turn change
        _check_xy(x, y)
        if piece not in (Black, White):
            raise ValueError("piece must be Black or White")
        bl, wh, _, r = _device().step(self._black, self._white, piece, x + 8 * y)
        if r <= 0:
            return 0
        self._set_bits(bl, wh)
        return r

    def put_s(self, stri):  # board.py:192-209
        code = codec.move_code(stri)  # raises IndexError for 'a9' like board.py:162
        bl, wh, _, r = _device().step(self._black, self._white, self.turn, code)
        if r >= 0:
            self._set_bits(bl, wh)
            self.nturn += 1
            self.turn = White if self.turn == Black else Black
        return r

    # ---------------------------------------------------------------- host-side helpers / codecs
    def str_from_turn(self, color):  # board.py:66-72
        return "Black" if color == Black else "White" if color == White else "None"

    def mask_count(self, color, mask):  # board.py:74-81
        bb = self._black if color == Black else self._white if color == White else \
            ~(self._black | self._white) & ((1 << 64) - 1)
        return bin(bb & mask & ((1 << 64) - 1)).count("1")

    @classmethod
    def show_mask(cls, mask):  # board.py:83-92
        q = cls()
        q._set_bits(mask & ((1 << 64) - 1), 0)
        print(q)

    def __str__(self):  # board.py:94-122
        ret = "  A B C D E F G H\n"
        for y in range(8):
            i = y + 1
            ret += str(i)
            for x in range(8):
                c = self.get(x, y)
                ret += " " + ("*" if c == 1 else "O" if c == 2 else ".")
            if i == 4:
                ret += "      " + self.str_from_turn(self.turn) + "'s turn"
            elif i == 5:
                ret += "      Black: " + str(self.n_black())
            elif i == 6:
                ret += "      White: " + str(self.n_white())
            ret += "\n"
        return ret

    def coord_from_handstr(self, handstr):  # board.py:176-185
        return codec.coord_from_handstr(handstr)

    def handstr_from_coord(self, x, y):  # board.py:187-190
        return codec.handstr_from_coord(x, y)

    def serialize_tuple(self):  # board.py:211-212
        return self.board, self.turn

    def serialize_str(self, append_turn=True):  # board.py:214-221
        return codec.serialize_str(self._black, self._white, self.turn, append_turn)

    def serialize_board(self):  # board.py:223-232
        return codec.serialize_board(self._black, self._white)

    def serialize_turn(self):  # board.py:234-235
        return codec.string_from_turn(self.turn)

    def string_from_turn(self, turn):  # board.py:237-243
        return codec.string_from_turn(turn)

    def turn_from_string(self, turn_string):  # board.py:245-251
        return codec.turn_from_string(turn_string)

    def deserialize(self, board_str, turn_str, nturn):  # board.py:253-262
        self._set_bits(*codec.deserialize_board(board_str, self._black, self._white))
        self.turn = codec.turn_from_string(turn_str)
        self.nturn = nturn


def is_within_board(x, y):  # board.py:265-266
    return 0 <= x < 8 and 0 <= y < 8


def clone_board(board):  # board.py:269-276
    return [[board[i][j] for j in range(8)] for i in range(8)]


def boards_to_numpy(boards):
    """list of Board -> (n, 2) uint64 array, for moving host games into a batch."""
    return np.array([b.bitboards() for b in boards], dtype=np.uint64).reshape(-1, 2)
