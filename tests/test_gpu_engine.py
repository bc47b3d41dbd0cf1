"""The Edax-protocol engine shim (subproc_amd.engine) driven exactly as the
reference's Player/GameRunner drive an engine (game_runner.py:9-201, restated
in Python 3 here: the reference is Python 2 and needs the external binaries)."""
import re
import subprocess
import sys

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

from subproc_amd import board as gboard  # noqa: E402
from subproc_amd import codec  # noqa: E402


class Player:  # game_runner.py:9-64 protocol
    def __init__(self, args):
        self.proc = subprocess.Popen([sys.executable, "-m", "subproc_amd.engine", *args], stdin=subprocess.PIPE,
                                     stdout=subprocess.PIPE, text=True, bufsize=1)
        self.name = ""

    def _w(self, s):
        self.proc.stdin.write(s)
        self.proc.stdin.flush()

    def go(self):
        self._w("go\n")
        out = "".join(self.proc.stdout.readline() for _ in range(3))
        out = re.sub(r"[\r\n]+", "", out)
        b = re.findall(r">(.+) plays [WB]?([a-zA-Z][0-9]|PS)", out.rstrip())
        self.name = b[0][0]
        return b[0][1]

    def init(self):
        self._w("init\n")
        self.proc.stdout.readline()

    def play(self, hand):
        self._w(hand + "\n")
        out = "".join(self.proc.stdout.readline() for _ in range(3))
        a = re.findall(r"(.+) play ([a-zA-Z][0-9]|PS|ps)", out.rstrip())
        return a[0][1]

    def show_hamlet_param(self):  # game_runner.py:66-73: 'verbose 0' is sent and never read
        self._w("verbose p\n")
        b = self.proc.stdout.readline().rstrip()
        self._w("verbose 0\n")
        return b

    def show(self):  # game_runner.py:75-102
        self._w("verbose 1\n")
        output = "".join(self.proc.stdout.readline() for _ in range(13))
        b = re.findall(r".*(Black|White|black|white) won.*", output.rstrip())
        self._w("verbose 0\n")
        a = re.findall(r".*(Game Over).*", self.proc.stdout.readline().rstrip())
        won = "None"
        if len(b) and len(b[0]):
            won = b[0]
        return len(a) > 0, won

    def end_process(self):
        self._w("quit\n")
        self.proc.stdout.readline()
        self.proc.communicate(timeout=60)


def play_a_game(black, white, end=True):  # game_runner.py:154-201 without randomisation
    black.init()
    white.init()
    b = gboard.Board()
    record = [b.serialize_str()]
    moves = []
    over = b.is_game_over()
    atk, dfn = black, white
    while not over:
        ha = atk.go().lower()
        assert b.put_s(ha) >= 0, ha
        moves.append(codec.move_code(ha))
        record.append(b.serialize_str())
        dfn.play(ha)
        over = b.is_game_over()
        atk, dfn = dfn, atk
    if end:
        black.end_process()
        white.end_process()
    return b, moves, record


@pytest.mark.parametrize("pa,pb", [("greedy", "random"), ("random", "random")])
def test_engine_plays_full_game(pa, pb):
    black = Player(["--policy", pa, "--name", "GPU-%s" % pa, "--seed", "1"])
    white = Player(["--policy", pb, "--name", "GPU-%s" % pb, "--seed", "2"])
    try:
        final, moves, record = play_a_game(black, white)
    finally:
        for p in (black, white):
            if p.proc.poll() is None:
                p.proc.kill()
    assert final.is_game_over()
    assert black.name == "GPU-%s" % pa
    # the game record replays bit-exactly through the oracle (board.py semantics)
    mv = np.full((1, 128), 255, np.uint8)
    mv[0, :len(moves)] = moves
    o = oracle.replay(mv, np.array([len(moves)], np.uint8))
    for k, line in enumerate(record):
        bl, wh = o["boards"][0, k]
        assert oracle.serialize_str(bl, wh, o["turn"][0, k]) == line
    assert o["end"][0, len(moves)] == 1


def test_engine_eval_choice_equals_kernel_policy(tmp_path):
    """--policy eval picks exactly what the kernels' eval policy picks (first
    move of an eval rollout with n_random = 0 from the same position), with the
    table read from a paramgen-format file."""
    from subproc_amd import engine, ops, params
    w = np.random.default_rng(21).integers(-127, 128, (4, 9)).astype(np.int8)
    path = tmp_path / "param.bin"
    params.write_paramgen(path, w)
    eng = engine.Engine(policy="eval", weights=params.read_paramgen(path)[1])
    pos = ops.sample_midgame(48, 77, device="cuda")
    r = ops.rollout(48, 5, 0, "eval", 0, start=pos.boards, start_turn=pos.turn, record_moves=True, weights=w,
                    device="cuda")
    first = r.moves[:, 0].cpu().tolist()
    bits = ops.to_numpy_u64(pos.boards)
    for i in range(48):
        eng.board = gboard.Board()
        eng.board._set_bits(int(bits[i, 0]), int(bits[i, 1]))
        eng.board.turn = int(pos.turn[i])
        assert codec.move_code(eng.choose().lower()) == first[i], i


def test_engine_eval_process_with_paramgen_file(tmp_path):
    from subproc_amd import params
    path = tmp_path / "param.bin"
    params.write_paramgen(path, params.DEFAULT_WEIGHTS)
    black = Player(["--policy", "eval", "--params", str(path), "--name", "GPU-eval"])
    white = Player(["--policy", "random", "--name", "GPU-random", "--seed", "3"])
    try:
        final, moves, record = play_a_game(black, white)
    finally:
        for p in (black, white):
            if p.proc.poll() is None:
                p.proc.kill()
    assert final.is_game_over() and black.name == "GPU-eval"


def test_engine_greedy_choice_equals_kernel_policy():
    """--policy greedy (all children in one oth_step launch, mobility from
    legal_next) picks exactly what the kernels' greedy policy picks: the first
    move of a greedy rollout with n_random = 0 from the same position."""
    from subproc_amd import engine, ops
    eng = engine.Engine(policy="greedy")
    n = 64
    pos = ops.sample_midgame(n, 78, device="cuda")
    r = ops.rollout(n, 5, 0, "greedy", 0, start=pos.boards, start_turn=pos.turn, record_moves=True, device="cuda")
    first = r.moves[:, 0].cpu().tolist()
    bits = ops.to_numpy_u64(pos.boards)
    for i in range(n):
        eng.board = gboard.Board()
        eng.board._set_bits(int(bits[i, 0]), int(bits[i, 1]))
        eng.board.turn = int(pos.turn[i])
        assert codec.move_code(eng.choose().lower()) == first[i], i


def test_engine_show_reports_the_winner():
    """Player.show() (game_runner.py:75-102) on the shim: (False, 'None')
    mid-game, (True, winner) once the game is over, where the winner is
    'Black' / 'White' by the final discs ('None' for a draw); the unread
    'verbose 0' of show_hamlet_param does not desync the protocol."""
    black = Player(["--policy", "greedy", "--name", "GPU-b", "--seed", "4"])
    white = Player(["--policy", "random", "--name", "GPU-w", "--seed", "5"])
    try:
        assert black.show_hamlet_param() == "GPU-b policy=greedy"
        black.init()
        assert black.show() == (False, "None")
        final, moves, record = play_a_game(black, white, end=False)
        nb, nw = final.n_black(), final.n_white()
        want = "Black" if nb > nw else ("White" if nw > nb else "None")
        assert black.show() == (True, want)
        assert white.show() == (True, want)
        assert "policy=random" in white.show_hamlet_param()
        assert white.show() == (True, want)
        black.end_process()
        white.end_process()
    finally:
        for p in (black, white):
            if p.proc.poll() is None:
                p.proc.kill()
