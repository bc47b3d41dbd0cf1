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

The positions come from the HIP replay kernel (``ops.replay``) and the text from
the HIP serializer (``ops.book_text``); only the file assembly (headers,
slicing per game) is host work.  Redis/DynamoDB I/O itself stays out of scope.
"""
import os

import torch

from . import ops
from ._lib import BOOK_LINE, POS_STRIDE


class GameBooks:
    """Books of n games played on the GPU (a rollout with ``record_moves=True``)."""

    def __init__(self, moves, plies, start=None, start_turn=None):
        self.plies = plies
        self.n = moves.shape[0]
        self.pos = ops.replay(moves, plies, start, start_turn)
        flat_b = self.pos.boards.view(-1, 2)
        flat_t = self.pos.turn.view(-1)
        self._text = ops.book_text(flat_b, flat_t)  # n * 129 lines, 67 bytes each
        self._plies_host = None

    @classmethod
    def from_rollout(cls, r, start=None, start_turn=None):
        if r.moves is None or r.plies is None:
            raise ValueError("rollout must be run with record_moves=True and want_plies=True")
        return cls(r.moves, r.plies, start, start_turn)

    def _plies(self):
        if self._plies_host is None:
            self._plies_host = self.plies.cpu().tolist()
        return self._plies_host

    def lines(self, g):
        """serialize_str() of every recorded board of game g (board.py:214-221)."""
        p = self._plies()[g]
        raw = self._text[g * POS_STRIDE * BOOK_LINE:(g * POS_STRIDE + p + 1) * BOOK_LINE].cpu().numpy().tobytes()
        return raw.decode("ascii").splitlines()

    def flat_file_bytes(self, g, black_name="gpu_black", white_name="gpu_white"):
        """Exactly the bytes FlatFileRecorder.store() writes (game_recorder.py:67-76)."""
        p = self._plies()[g]
        body = self._text[g * POS_STRIDE * BOOK_LINE:(g * POS_STRIDE + p + 1) * BOOK_LINE].cpu().numpy().tobytes()
        return ("%% Black: %s\n%% White: %s\n" % (black_name, white_name)).encode("ascii") + body

    def write_flat_files(self, out_dir, title="gpu", black_name="gpu_black", white_name="gpu_white", games=None):
        """One FlatFileRecorder-format file per game: <out_dir>/<title>_<g>."""
        os.makedirs(out_dir, exist_ok=True)
        games = range(self.n) if games is None else games
        text = self._text.cpu().numpy()
        pl = self._plies()
        paths = []
        for g in games:
            body = text[g * POS_STRIDE * BOOK_LINE:(g * POS_STRIDE + pl[g] + 1) * BOOK_LINE].tobytes()
            path = os.path.join(out_dir, "%s_%d" % (title, g))
            with open(path, "wb") as f:
                f.write(("%% Black: %s\n%% White: %s\n" % (black_name, white_name)).encode("ascii"))
                f.write(body)
            paths.append(path)
        return paths

    def records(self, g):
        """RedisRecorder.add() dicts of game g, in recording order."""
        p = self._plies()[g]
        end = self.pos.end[g, :p + 1].cpu().tolist()
        out = []
        for k, line in enumerate(self.lines(g)):
            out.append({"book": line[:64], "whosturn": line[65], "turn": k, "end": bool(end[k])})
        return out

    def features(self, side):
        """counts() features (ops.features) of every recorded position for side
        1 ('O') or 2 ('X'): (n, 129, 10) uint8; rows past plies are undefined."""
        flat = self.pos.boards.view(-1, 2)
        sd = torch.full((flat.shape[0],), side, dtype=torch.uint8, device=flat.device)
        return ops.features(flat, sd).view(self.n, POS_STRIDE, -1)
