"""Book emitter: GPU self-play written in the reference's
book record formats, so replearn.learn_books (replearn.py:27-46) and the
learners consume GPU games unchanged.

* Flat file (FlatFileRecorder, game_recorder.py:41-79): two header lines
  "% Black: <name>" / "% White: <name>", then one Board.serialize_str() line
  per recorded board.  The board is recorded after Board() and after every
  put_s (game_runner.py:169-184), so a game of `plies` env-steps has plies + 1
  lines.
* Per-ply records (RedisRecorder.add / DynamoDBRecorder.add,
  game_recorder.py:107-114, 197-205): {'book': serialize_board(),
  'whosturn': serialize_turn(), 'turn': nturn, 'end': is_game_over()}.

The positions come from the HIP replay kernel (``ops.replay_rows``) and the text from
the HIP serializer (``ops.book_text``); only the file assembly (headers,
slicing per game) is host work.  Redis/DynamoDB I/O itself stays out of scope.

The reader's side (books from any source, e.g. the reference's own Edax
matches): ``parse_book_strings`` turns records' board strings into bitboards
with the HIP parser (``ops.book_parse``, board_from_a_book of parameter.py:5-8)
and ``read_flat_file`` a FlatFileRecorder file; td.StateMap.update_from_records
feeds such books to the learner.
"""
import os

import numpy as np
import torch

from . import codec, ops
from ._lib import BOOK_LINE, MOVES_STRIDE

# Board() (board.py:22-27) as serialize_board writes it: Board.deserialize
# writes a string over a fresh Board, so the squares a short string does not
# reach keep these characters
_OPEN_BLACK, _OPEN_WHITE = 0x0000000810000000, 0x0000001008000000
OPENING_BOOK = codec.serialize_board(_OPEN_BLACK, _OPEN_WHITE)


def pack_book_strings(strings):
    """The 64 bytes Board.deserialize reads from each board string onto a
    fresh Board (board.py:253-258), concatenated (numpy uint8, 64 per string):
    a string of 64 characters as it is; a shorter one completed with the
    opening's characters for the squares it does not reach; a longer one raises
    IndexError as the reference does (its 65th character indexes row 8).  Any
    character other than 'O' and 'X' reads as Empty (turn_from_string), so a
    character outside latin-1 is stored as '?'."""
    parts = []
    for s in strings:
        if len(s) > 64:
            raise IndexError("list index out of range")
        parts.append(s if len(s) == 64 else s + OPENING_BOOK[len(s):])
    return np.frombuffer("".join(parts).encode("latin-1", "replace"), dtype=np.uint8)


def parse_book_strings(strings, device="cuda"):
    """board_from_a_book's board (parameter.py:5-8) of each string, parsed on
    the GPU: (n, 2) int64 [black, white] on ``device``."""
    packed = pack_book_strings(strings)
    n = packed.size // 64
    if n == 0:
        return torch.empty((0, 2), dtype=torch.int64, device=device)
    text = torch.from_numpy(packed.copy()).to(device)
    return ops.book_parse(text, n)[0]


def read_flat_file(path, device="cuda"):
    """A FlatFileRecorder file (game_recorder.py:67-76) back into the game:
    returns (black_name, white_name, boards (n, 2) int64, turn (n,) uint8) on
    ``device``, the body's serialize_str lines parsed in place by the HIP
    parser (stride OTH_BOOK_LINE)."""
    with open(path, "rb") as f:
        data = f.read()
    head = []
    for _ in range(2):
        nl = data.index(b"\n")
        head.append(data[:nl].decode("latin-1"))
        data = data[nl + 1:]
    names = []
    for line, tag in zip(head, ("% Black: ", "% White: ")):
        if not line.startswith(tag):
            raise ValueError("not a FlatFileRecorder file: %r" % line)
        names.append(line[len(tag):])
    if len(data) % BOOK_LINE:
        raise ValueError("the body is not a whole number of %d-byte serialize_str lines" % BOOK_LINE)
    n = len(data) // BOOK_LINE
    if n == 0:
        return names[0], names[1], torch.empty((0, 2), dtype=torch.int64, device=device), \
            torch.empty(0, dtype=torch.uint8, device=device)
    text = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to(device)
    boards, turn = ops.book_parse(text, n, stride=BOOK_LINE, want_turn=True)
    return names[0], names[1], boards, turn


class GameBooks:
    """Books of n games played on the GPU (a rollout with ``record_moves=True``).

    The recorded positions are replayed into packed rows (``ops.replay_rows``:
    game g's boards are rows ``row_off[g] .. row_off[g] + plies[g]``) and the
    text is serialised over exactly those rows, so neither kernel touches the
    unused tail of a 129-row stride."""

    def __init__(self, moves, plies, start=None, start_turn=None):
        self.plies = plies
        self.n = moves.shape[0]
        self.pos = ops.replay_rows(moves, plies, start, start_turn)
        self._text = ops.book_text(self.pos.boards, self.pos.turn)  # one 67-byte line per recorded board
        self._plies_host = None
        self._off_host = None

    @classmethod
    def from_rollout(cls, r, start=None, start_turn=None):
        if r.moves is None or r.plies is None:
            raise ValueError("rollout must be run with record_moves=True and want_plies=True")
        return cls(r.moves, r.plies, start, start_turn)

    def _plies(self):
        if self._plies_host is None:
            self._plies_host = [min(p, MOVES_STRIDE) for p in self.plies.cpu().tolist()]
        return self._plies_host

    def _rows(self, g):
        """(first row, row count) of game g in the packed tables."""
        if self._off_host is None:
            self._off_host = self.pos.row_off.cpu().tolist()
        return self._off_host[g], self._plies()[g] + 1

    def _body(self, g):
        r0, k = self._rows(g)
        return self._text[r0 * BOOK_LINE:(r0 + k) * BOOK_LINE].cpu().numpy().tobytes()

    def lines(self, g):
        """serialize_str() of every recorded board of game g (board.py:214-221)."""
        return self._body(g).decode("ascii").splitlines()

    def flat_file_bytes(self, g, black_name="gpu_black", white_name="gpu_white"):
        """Exactly the bytes FlatFileRecorder.store() writes (game_recorder.py:67-76)."""
        return ("%% Black: %s\n%% White: %s\n" % (black_name, white_name)).encode("ascii") + self._body(g)

    def write_flat_files(self, out_dir, title="gpu", black_name="gpu_black", white_name="gpu_white", games=None):
        """One FlatFileRecorder-format file per game: <out_dir>/<title>_<g>."""
        os.makedirs(out_dir, exist_ok=True)
        games = range(self.n) if games is None else games
        text = self._text.cpu().numpy()
        paths = []
        for g in games:
            r0, k = self._rows(g)
            body = text[r0 * BOOK_LINE:(r0 + k) * BOOK_LINE].tobytes()
            path = os.path.join(out_dir, "%s_%d" % (title, g))
            with open(path, "wb") as f:
                f.write(("%% Black: %s\n%% White: %s\n" % (black_name, white_name)).encode("ascii"))
                f.write(body)
            paths.append(path)
        return paths

    def records(self, g):
        """RedisRecorder.add() dicts of game g, in recording order."""
        r0, k = self._rows(g)
        end = self.pos.end[r0:r0 + k].cpu().tolist()
        return [{"book": line[:64], "whosturn": line[65], "turn": p, "end": bool(end[p])}
                for p, line in enumerate(self.lines(g))]

    def features(self, side):
        """counts() features (ops.features) of every recorded position for side
        1 ('O') or 2 ('X'): (R, 10) uint8 in the packed row order (game g's
        positions are rows ``game_rows(g)``)."""
        flat = self.pos.boards
        sd = torch.full((flat.shape[0],), side, dtype=torch.uint8, device=flat.device)
        return ops.features(flat, sd)

    def game_rows(self, g):
        """The slice of game g's rows in pos / features / the text lines."""
        r0, k = self._rows(g)
        return slice(r0, r0 + k)
