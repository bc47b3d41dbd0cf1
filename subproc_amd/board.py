"""Drop-in ``board`` module: the reference ``Board`` class API (board.py:20-276)
served by the MI355X kernels.

Callers of the reference (game_runner.py:3, learn_base.py:1, parameter.py:2)
run unchanged with ``sys.modules['board'] = subproc_amd.board``.
Same method names, argument order, colour values (Empty 0, Black 1, White 2),
return codes, Edax move strings -- and the same answers on every input
board.py accepts, including the ones its plain-list implementation lets
through:

* the side to move (or a ``piece``) may be Empty or any other value:
  hostile(piece) is Black unless piece is Black (board.py:155-159), so with
  Empty to move the Black runs that end on an empty square are "flipped" to
  Empty, and ``put_s`` then hands the turn to Black (205-208);
* coordinates index ``board[y][x]`` like Python lists: -8..-1 wrap for the
  emptiness test and the placed piece, while the ray scan starts from the
  coordinate as given (an off-board origin next to the edge scans into the
  board); ``hands_for_direc`` takes any origin and any direction;
* ``board`` is a live ``board[y][x]`` view: writing through it changes the
  game, as writing into board.py's list-of-lists does;
* a square may hold a value other than Empty/Black/White (``set``): it then
  blocks rays like board.py's cell would and ends the runs of a piece equal
  to it.

The rules -- legal moves, flips, pass/terminal, disc counts -- are computed by
the HIP library (one batch-of-one launch per call, through subproc_amd.ops):
``oth_legal`` / ``oth_step`` / ``oth_result`` for a board of Black, White and
empty squares, ``oth_hands`` (any origin, any direction, any own/hostile
squares) for the rest.  This class keeps the two bitboards, any other cell
values, the side to move and the ply counter on the host, plus the text
codecs.  For throughput use :class:`subproc_amd.env.VecEnv` / :mod:`subproc_amd.ops`.
"""
import operator
import threading

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
_M64 = (1 << 64) - 1
_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1


def _i64(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def _u64(x):
    return x & _M64


def _popcount(x):
    return bin(x & _M64).count("1")


def _side_code(piece):
    """The C-ABI side code of a piece value (include/othello.h): 1 / 2 / 0, and
    3 for a value equal to none of them (a piece no square of a Black/White/
    Empty board holds).  Decided with board.py's own == comparisons."""
    if piece == Black:
        return Black
    if piece == White:
        return White
    if piece == Empty:
        return Empty
    return 3


class _Device:
    """The HIP library for batch-of-one calls: fixed pinned / device staging
    buffers, raw C-ABI launches on torch's current stream, one host sync per
    call, and an analysis cache.

    A GameRunner ply asks puttables(turn), put_s and is_game_over
    (game_runner.py:137-158).  ``step`` therefore also analyses the position it
    produces -- both sides' legal masks, disc counts, is_game_over -- in the
    same sync (oth_step, 2 x oth_legal, oth_result), and the next questions
    about that position are answered from the cache: one sync per ply.

    Staging layout (int64 words; byte offsets for the uint8 arguments):
      in : [0] black [1] white | byte 16 side code, 17 move, 18 = 1, 19 = 2
      out: [0] black [1] white (step result) | [2] legal Black [3] legal White
           [4] flips | byte 40 ret, 41 n_black, 42 n_white, 43 is_game_over
    """

    _CACHE_MAX = 1 << 16

    def __init__(self):
        import torch

        from . import _lib

        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.OthelloLibraryError("subproc_amd.board needs a ROCm GPU: there is no CPU path")
        self.torch = torch
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.hin = torch.zeros(4, dtype=torch.int64).pin_memory()
        self.hout = torch.zeros(6, dtype=torch.int64).pin_memory()
        self.din = torch.zeros(4, dtype=torch.int64, device=self.dev)
        self.dout = torch.zeros(6, dtype=torch.int64, device=self.dev)
        self.hin_w = self.hin.numpy()
        self.hin_b = self.hin_w.view(np.uint8)
        self.hout_w = self.hout.numpy().view(np.uint64)
        self.hout_b = self.hout_w.view(np.uint8)
        self.hin_b[18], self.hin_b[19] = Black, White
        self.i, self.o = self.din.data_ptr(), self.dout.data_ptr()
        self.cache = {}
        self._check = _lib.check

    def _launch_in(self, black, white, code=0, move=0):
        self.hin_w[0], self.hin_w[1] = _i64(black), _i64(white)
        self.hin_b[16], self.hin_b[17] = code, move
        self.din.copy_(self.hin, non_blocking=True)
        return self.torch.cuda.current_stream().cuda_stream

    def _analyse_on_device(self, boards_ptr, s):
        L, o, i = self.lib, self.o, self.i
        self._check(L.oth_legal(boards_ptr, i + 18, o + 16, 1, s), "oth_legal")
        self._check(L.oth_legal(boards_ptr, i + 19, o + 24, 1, s), "oth_legal")
        self._check(L.oth_result(boards_ptr, o + 41, o + 42, None, o + 43, 1, s), "oth_result")

    def _fetch(self):
        self.hout.copy_(self.dout, non_blocking=True)
        self.torch.cuda.current_stream().synchronize()
        w, b = self.hout_w, self.hout_b
        return int(w[0]), int(w[1]), (int(w[2]), int(w[3]), int(b[41]), int(b[42]), bool(b[43])), int(w[4]), int(
            b.view(np.int8)[40])

    def _remember(self, key, analysis):
        if len(self.cache) >= self._CACHE_MAX:
            self.cache.clear()
        self.cache[key] = analysis

    def analyse(self, black, white):
        """(legal Black, legal White, n_black, n_white, is_game_over) of a
        board of Black, White and empty squares (board.py:37-58)."""
        key = (black, white)
        a = self.cache.get(key)
        if a is None:
            s = self._launch_in(black, white)
            self._analyse_on_device(self.i, s)
            a = self._fetch()[2]
            self._remember(key, a)
        return a

    def legal(self, black, white, code):
        """puttables(piece) as a mask for any side code (oth_legal)."""
        if code in (Black, White):
            return self.analyse(black, white)[code - 1]
        s = self._launch_in(black, white, code)
        self._check(self.lib.oth_legal(self.i, self.i + 16, self.o + 16, 1, s), "oth_legal")
        return self._fetch()[2][0]

    def result(self, black, white):
        a = self.analyse(black, white)
        return a[2], a[3], a[4]

    def step(self, black, white, code, move):
        """put_s (oth_step) -> (black, white, flips, ret); the position it
        leaves is analysed in the same sync."""
        s = self._launch_in(black, white, code, move)
        L, i, o = self.lib, self.i, self.o
        self._check(L.oth_step(i, i + 16, i + 17, o, None, o + 32, None, o + 40, None, 1, s), "oth_step")
        self._analyse_on_device(o, s)
        bl, wh, a, flips, ret = self._fetch()
        self._remember((bl, wh), a)
        return bl, wh, flips, ret

    def hands(self, own, hostile, rows):
        """rows: [(x, y, dx, dy), ...] with one own/hostile pair -> run lengths."""
        from . import ops

        t = self.torch
        n = len(rows)
        a = t.tensor([[_i64(own), _i64(hostile), *r] for r in rows], dtype=t.int64).t().contiguous()
        a = a.pin_memory().to(self.dev, non_blocking=True)
        out = ops.hands(a[0].contiguous(), a[1].contiguous(), a[2].contiguous(), a[3].contiguous(),
                        a[4].contiguous(), a[5].contiguous())
        return out.cpu().tolist()[:n]


_TLS = threading.local()


def _device():
    """This thread's _Device: every call stages through the object's pinned and
    device buffers between its launch and its fetch, so Boards used from
    several threads each get their own (reference Boards share no state)."""
    d = getattr(_TLS, "dev", None)
    if d is None:
        d = _TLS.dev = _Device()
    return d


def _index(i):
    """A list index as board.py's ``board[y][x]`` takes it: integers (or
    __index__ objects) in -8..7, negative ones wrapping; else IndexError."""
    i = operator.index(i)
    if not -8 <= i < 8:
        raise IndexError("list index out of range")
    return i % 8


def _coord(c):
    """An origin / direction component for the scan: any integer (bounded to
    int64: every value past that is far off the board, and so is the bound)."""
    c = operator.index(c)
    return min(max(c, _I64_MIN), _I64_MAX)


class _Row:
    """``board[y]``: a live row of the board (board.py:23's inner list)."""

    __slots__ = ("_b", "_y")

    def __init__(self, b, y):
        self._b, self._y = b, y

    def __len__(self):
        return 8

    def __getitem__(self, x):
        if isinstance(x, slice):
            return [self._b._cell(i + 8 * self._y) for i in range(8)][x]
        return self._b._cell(_index(x) + 8 * self._y)

    def __setitem__(self, x, v):
        if isinstance(x, slice):
            xs = range(8)[x]
            vs = list(v)
            if len(vs) != len(xs):
                raise ValueError("a board row has 8 squares: a slice assignment must keep its length")
            for i, c in zip(xs, vs):
                self._b._set_cell(i + 8 * self._y, c)
            return
        self._b._set_cell(_index(x) + 8 * self._y, v)

    def __iter__(self):
        return iter(self[:])

    def __eq__(self, other):
        try:
            return list(self) == list(other)
        except TypeError:
            return NotImplemented

    def __repr__(self):
        return repr(list(self))


class _Rows:
    """``board``: the live list-of-lists view ``board[y][x]`` (board.py:23)."""

    __slots__ = ("_b",)

    def __init__(self, b):
        self._b = b

    def __len__(self):
        return 8

    def __getitem__(self, y):
        if isinstance(y, slice):
            return [_Row(self._b, i) for i in range(8)[y]]
        return _Row(self._b, _index(y))

    def __setitem__(self, y, row):
        if isinstance(y, slice):
            ys = range(8)[y]
            rows = list(row)
            if len(rows) != len(ys):
                raise ValueError("the board has 8 rows: a slice assignment must keep its length")
            for i, r in zip(ys, rows):
                self[i] = r
            return
        cells = list(row)
        if len(cells) != 8:
            raise ValueError("a board row has 8 squares")
        _Row(self._b, _index(y))[:] = cells

    def __iter__(self):
        return (_Row(self._b, i) for i in range(8))

    def __eq__(self, other):
        try:
            return [list(r) for r in self] == [list(r) for r in other]
        except TypeError:
            return NotImplemented

    def __repr__(self):
        return repr([list(r) for r in self])


class Board:
    """board.py:20 -- one game; the rules run on the GPU."""

    def __init__(self):  # board.py:22-27
        self._black = _OPEN_BLACK
        self._white = _OPEN_WHITE
        self._other = {}  # square -> a value equal to none of Empty/Black/White
        self.turn = Black
        self.nturn = 0
        self._cache = {}

    # ---------------------------------------------------------------- state
    @property
    def board(self):
        """The live ``board[y][x]`` view (board.py:23): reads and writes go to this game."""
        return _Rows(self)

    @board.setter
    def board(self, rows):
        rows = list(rows)
        if len(rows) != 8:
            raise ValueError("the board has 8 rows")
        _Rows(self)[:] = rows

    def _cell(self, sq):
        if sq in self._other:
            return self._other[sq]
        return Black if self._black >> sq & 1 else White if self._white >> sq & 1 else Empty

    def _set_cell(self, sq, piece):
        bit = 1 << sq
        bl, wh = self._black & ~bit, self._white & ~bit
        self._other.pop(sq, None)
        code = _side_code(piece)
        if code == Black:
            bl |= bit
        elif code == White:
            wh |= bit
        elif code == 3:
            self._other[sq] = piece
        self._set_bits(bl, wh)

    def _set_bits(self, black, white):
        self._black, self._white = black, white
        self._cache.clear()

    def bitboards(self):
        """(black, white) uint64 bitboards, sq = x + 8*y."""
        return self._black, self._white

    def set(self, piece, x, y):  # board.py:60-61
        self._set_cell(self._sq(x, y), piece)

    def get(self, x, y):  # board.py:63-64
        return self._cell(self._sq(x, y))

    @staticmethod
    def _sq(x, y):
        # board[y][x]: the row index is taken first, as Python evaluates it
        yy = _index(y)
        return _index(x) + 8 * yy

    # ---------------------------------------------------------------- own / hostile squares of a piece
    def _empty_mask(self):
        occ = self._black | self._white
        for sq in self._other:
            occ |= 1 << sq
        return ~occ & _M64

    def _masks(self, piece):
        """(own, hostile): the squares holding `piece` and hostile(piece) (board.py:155-159)."""
        hostile = self._white if piece == Black else self._black
        if piece == Black:
            own = self._black
        elif piece == White:
            own = self._white
        elif piece == Empty:
            own = self._empty_mask()
        else:
            own = 0
        for sq, v in self._other.items():
            if v == piece:
                own |= 1 << sq
        return own, hostile

    def _fast(self, piece):
        """The board-of-three-values path (oth_legal / oth_step) applies."""
        return not self._other

    # ---------------------------------------------------------------- GPU-backed rules
    def _result(self):
        return _device().result(self._black, self._white)

    def _legal(self, piece):
        code = _side_code(piece)
        if self._fast(piece):
            if code in (Black, White):
                return _device().legal(self._black, self._white, code)  # the device caches the analysis
            k = ("legal", self._black, self._white, code)
            if k not in self._cache:
                self._cache[k] = _device().legal(self._black, self._white, code)
            return self._cache[k]
        # a board holding other values: every square's 8 rays through oth_hands
        own, hostile = self._masks(piece)
        rows = [(sq % 8, sq // 8, dx, dy) for sq in range(64) for (dx, dy) in DIRECS]
        runs = _device().hands(own, hostile, rows)
        empty = self._empty_mask()
        m = 0
        for sq in range(64):
            if empty >> sq & 1 and any(runs[8 * sq:8 * sq + 8]):
                m |= 1 << sq
        return m

    def count_over_board(self, fun):  # board.py:29-35
        return sum(1 for y in range(8) for x in range(8) if fun(self.get(x, y)))

    def n_black(self):  # board.py:37-38
        return self._result()[0]

    def n_white(self):  # board.py:40-41
        return self._result()[1]

    def n_empty(self):  # board.py:43-44
        nb, nw, _ = self._result()
        return 64 - nb - nw - len(self._other)

    def puttables(self, piece):  # board.py:46-52 (row-major == LSB-first)
        m = self._legal(piece)
        out = []
        while m:
            sq = (m & -m).bit_length() - 1
            out.append((sq % 8, sq // 8))
            m &= m - 1
        return out

    def n_puttable_for(self, piece):  # board.py:54-55
        return _popcount(self._legal(piece))

    def is_game_over(self):  # board.py:57-58
        if self._fast(None):
            return self._result()[2]
        return self.n_puttable_for(Black) == 0 and self.n_puttable_for(White) == 0

    def _runs(self, piece, x, y, direcs):
        own, hostile = self._masks(piece)
        return _device().hands(own, hostile, [(_coord(x), _coord(y), _coord(d[0]), _coord(d[1])) for d in direcs])

    def is_puttable_at(self, piece, x, y):  # board.py:141-149
        if self.get(x, y) != Empty:
            return False
        if self._fast(piece) and 0 <= x < 8 and 0 <= y < 8:
            return bool(self._legal(piece) >> (x + 8 * y) & 1)
        return sum(self._runs(piece, x, y, DIRECS)) > 0

    def hands_for_direc(self, direc, piece, x, y):  # board.py:124-139
        """[(piece, nx, ny), ...] captured along `direc` from (x, y): the run
        length from oth_hands, the squares are its first steps."""
        dx, dy = direc[0], direc[1]
        k = self._runs(piece, x, y, [(dx, dy)])[0]
        return [(piece, x + i * dx, y + i * dy) for i in range(1, k + 1)]

    def set_hands(self, hands):  # board.py:151-153
        for (piece, x, y) in hands:
            self.set(piece, x, y)

    def hostile(self, piece):  # board.py:155-159
        return White if piece == Black else Black

    def put(self, piece, x, y):  # board.py:161-174 -- flips, no turn change
        if self.get(x, y) != Empty:
            return 0
        if self._fast(piece) and 0 <= x < 8 and 0 <= y < 8:
            bl, wh, _, r = _device().step(self._black, self._white, _side_code(piece), x + 8 * y)
            if r <= 0:
                return 0
            self._set_bits(bl, wh)
            return r
        # an off-board origin or a board holding other values: direction by
        # direction as board.py does, the runs from oth_hands.  The rays are
        # disjoint, but from an off-board origin the square set(piece, x, y)
        # writes (board[y][x], wrapped) can lie on a later ray, so the rays
        # after a placement are scanned again on the updated board.
        count = 0
        runs = self._runs(piece, x, y, DIRECS)
        for d, (dx, dy) in enumerate(DIRECS):
            k = runs[d]
            if k:
                for i in range(1, k + 1):
                    self.set(piece, x + i * dx, y + i * dy)  # set_hands
                count += k
                self.set(piece, x, y)
                if d < 7:
                    runs[d + 1:] = self._runs(piece, x, y, DIRECS[d + 1:])
        return count

    def put_s(self, stri):  # board.py:192-209
        code = codec.move_code(stri)  # raises IndexError for 'a9' like board.py:162
        if self._fast(self.turn):
            bl, wh, _, r = _device().step(self._black, self._white, _side_code(self.turn), code)
            if r >= 0:
                self._set_bits(bl, wh)
        elif code == codec.PASS:
            r = 0
        elif code < 64:
            r = self.put(self.turn, code % 8, code // 8)
            r = -1 if r == 0 else r
        else:
            r = -1
        if r >= 0:
            self.nturn += 1
            self.turn = White if self.turn == Black else Black
        return r

    # ---------------------------------------------------------------- host-side helpers / codecs
    def str_from_turn(self, color):  # board.py:66-72
        return "Black" if color == Black else "White" if color == White else "None"

    def mask_count(self, color, mask):  # board.py:74-81
        if color == Black:
            bb = self._black
        elif color == White:
            bb = self._white
        elif color == Empty:
            bb = self._empty_mask()
        else:
            bb = 0
        for sq, v in self._other.items():
            if v == color:
                bb |= 1 << sq
        return _popcount(bb & mask)

    @classmethod
    def show_mask(cls, mask):  # board.py:83-92
        q = cls()
        q._set_bits(mask & _M64, 0)
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
        # cell i sets square (i % 8, i // 8); a 65th cell raises IndexError
        # after the first 64 were set, as board.py's set(cell, 0, 8) does
        for i, s in enumerate(board_str):
            if i >= 64:
                raise IndexError("list index out of range")
            self._set_cell(i, codec.turn_from_string(s))
        self.turn = codec.turn_from_string(turn_str)
        self.nturn = nturn


def is_within_board(x, y):  # board.py:265-266
    return 0 <= x < 8 and 0 <= y < 8


def clone_board(board):  # board.py:269-276
    return [[board[i][j] for j in range(8)] for i in range(8)]


def boards_to_numpy(boards):
    """list of Board -> (n, 2) uint64 array, for moving host games into a batch."""
    return np.array([b.bitboards() for b in boards], dtype=np.uint64).reshape(-1, 2)
