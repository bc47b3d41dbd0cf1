"""Edax-protocol engine backed by the GPU env.

The reference drives external engines through pipes with the Player class
(game_runner.py:9-102).  This module answers exactly the commands Player sends,
so ``proc_a_path = python -m subproc_amd.engine --policy greedy`` plugs a GPU
policy into GameRunner unchanged:

  init          -> 1 line                                   (game_runner.py:35-39)
  go            -> 3 lines; joined they match
                   ">(.+) plays [WB]?([a-zA-Z][0-9]|PS)"     (game_runner.py:19-33)
                   and the engine plays that move on its board
  <move>        -> 3 lines matching "(.+) play ([a-zA-Z][0-9]|PS|ps)"  (game_runner.py:41-54);
                   the move ('d3', 'ps', ...) is applied for the side to move
                   (go_for also sends the engine its OWN randomised moves, 149)
  verbose p     -> 1 line (parameter description)           (game_runner.py:66-73)
  verbose 1     -> 13 lines: the board display, the last line "Black won" /
                   "White won" once the game is over with a winner
                   (Player.show parses "(Black|White) won", game_runner.py:75-91)
  verbose 0     -> after a "verbose 1": 1 line, "Game Over" once the game is
                   over (Player.show reads one line and looks for it, 92-95);
                   otherwise nothing (show_hamlet_param sends it unread, 70)
  quit          -> 1 line, exit                              (game_runner.py:56-64)

Rules and move generation run on the GPU through the drop-in Board
(subproc_amd.board); the move choice is the env's policy: "random" (uniform
over legal moves, seeded), "greedy" (minimise the opponent's mobility, ties
to the first move in puttables order) or "eval" (maximise the mover's linear
eval of the child under an eval table, ties likewise -- the kernels' eval
policy).  ``--params FILE`` loads the table from the file paramgen.py writes
(paramgen.py:12-19), the file the reference's own engines read.
"""
import argparse
import random
import sys

import numpy as np
import torch

from . import board as gboard
from . import ops, params
from .codec import handstr_from_coord


class Engine:
    def __init__(self, name="GPU", policy="greedy", seed=0, weights=None):
        self.name = name
        self.policy = policy
        self.rng = random.Random(seed)
        self.weights = params.as_weights(params.DEFAULT_WEIGHTS if weights is None else weights)
        self.board = gboard.Board()
        self._shown = False  # a "verbose 1" awaits its "verbose 0" line

    def _children(self, puts, want_legal):
        """Every child of the side to move in ONE oth_step launch (board
        repeated per legal square): the StepResult on the device."""
        b = self.board
        bl, wh = b.bitboards()
        n = len(puts)
        dev = torch.device("cuda", torch.cuda.current_device())
        boards = ops.from_numpy_u64(np.array([[bl, wh]] * n, np.uint64), dev)
        side = torch.full((n,), b.turn, dtype=torch.uint8, device=dev)
        sq = torch.tensor([x + 8 * y for (x, y) in puts], dtype=torch.uint8, device=dev)
        return ops.step(boards, side, sq, want_flips=False, want_legal=want_legal), side

    def _choose_eval(self, puts):
        """The children's evals in one more oth_eval launch."""
        r, side = self._children(puts, want_legal=False)
        ev = ops.evaluate(r.boards, side, self.weights).cpu().tolist()
        k = max(range(len(puts)), key=lambda i: (ev[i], -i))  # puts is LSB-first: ties -> lowest square
        return handstr_from_coord(*puts[k])

    def _choose_greedy(self, puts):
        """A legal move hands the turn over, so each child's legal_next is the
        opponent's puttables: its popcount is n_puttable_for(hostile)."""
        r, _ = self._children(puts, want_legal=True)
        mob = [bin(v & (2**64 - 1)).count("1") for v in r.legal_next.cpu().tolist()]
        k = min(range(len(puts)), key=lambda i: (mob[i], i))  # ties -> lowest square
        return handstr_from_coord(*puts[k])

    def choose(self):
        b = self.board
        puts = b.puttables(b.turn)
        if not puts:
            return "PS"
        if self.policy == "random":
            x, y = puts[self.rng.randrange(len(puts))]
            return handstr_from_coord(x, y)
        if self.policy == "eval":
            return self._choose_eval(puts)
        return self._choose_greedy(puts)

    def handle(self, line, out):
        cmd = line.strip()
        if cmd == "init":
            self.board = gboard.Board()
            out("init done")
        elif cmd == "go":
            mv = self.choose()
            color = "B" if self.board.turn == gboard.Black else "W"
            self.board.put_s(mv.lower() if mv != "PS" else "PS")
            out("")
            out(">%s plays %s%s" % (self.name, color, mv.upper() if mv != "PS" else "PS"))
            out("")
        elif cmd == "verbose p":
            extra = " weights=%s" % self.weights.reshape(-1).tolist() if self.policy == "eval" else ""
            out("%s policy=%s%s" % (self.name, self.policy, extra))
        elif cmd == "verbose 1":
            b = self.board
            text = str(b).rstrip("\n").split("\n")[:12]
            text += [""] * (12 - len(text))
            won = ""
            if b.is_game_over() and b.n_black() != b.n_white():
                won = "Black won" if b.n_black() > b.n_white() else "White won"
            for t in text + [won]:
                out(t)
            self._shown = True
        elif cmd == "verbose 0":
            if self._shown:
                out("Game Over" if self.board.is_game_over() else "")
            self._shown = False
        elif cmd.startswith("verbose"):
            self._shown = False
        elif cmd == "quit":
            out("bye")
            return False
        elif cmd:
            mv = cmd.split()[-1]
            self.board.put_s(mv)
            out("")
            out("%s play %s" % (self.name, mv))
            out("")
        return True


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    p.add_argument("--name", default="GPU")
    p.add_argument("--policy", choices=["random", "greedy", "eval"], default="greedy")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--params", default=None, help="eval table in the paramgen.py file format (policy eval)")
    a = p.parse_args(argv)
    weights = params.read_paramgen(a.params)[1] if a.params else None
    eng = Engine(a.name, a.policy, a.seed, weights)

    def out(s):
        sys.stdout.write(s + "\n")
        sys.stdout.flush()

    for line in sys.stdin:
        if not eng.handle(line, out):
            break
    return 0


if __name__ == "__main__":
    sys.exit(main())
