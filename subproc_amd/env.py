"""Batched env API of the reference's env driver — reset / legal_moves / step /
result — over N games resident in HBM.

The reference drives one game per process (game_runner.py:154-201: Board(),
puttables, put_s, is_game_over, n_black/n_white); VecEnv keeps the same
per-game semantics for N games at once, each call one HIP launch on torch's
current stream.  State layout: boards (N,2) int64 bit
patterns [black, white], turn (N,) uint8, nturn (N,) uint8.
"""
import torch

from . import codec, ops


class VecEnv:
    def __init__(self, n, device="cuda"):
        if n <= 0:
            raise ValueError("n must be positive")
        self.n = n
        self.device = torch.device(device)
        self.boards, self.turn, self.nturn = ops.reset(n, self.device)

    # reference: Board() per game (game_runner.py:169)
    def reset(self, mask=None):
        """Reset every game, or only those where the bool tensor `mask` is set."""
        b, t, nt = ops.reset(self.n, self.device)
        if mask is None:
            self.boards, self.turn, self.nturn = b, t, nt
        else:
            self.boards = torch.where(mask[:, None], b, self.boards)
            self.turn = torch.where(mask, t, self.turn)
            self.nturn = torch.where(mask, nt, self.nturn)
        return self.boards, self.turn

    # reference: puttables(turn) (game_runner.py:137)
    def legal_moves(self):
        return ops.legal(self.boards, self.turn)

    # reference: put_s(hand) (game_runner.py:157)
    def step(self, moves):
        """Apply one move code per game (uint8: 0..63, 64 = pass) in place.
        Returns (ret int8, flips int64, legal_next int64) where ret follows
        board.put_s: -1 illegal/unchanged, 0 pass, n >= 1 discs flipped."""
        if moves.dtype != torch.uint8:
            moves = moves.to(torch.uint8)
        r = ops.step(self.boards, self.turn, moves.contiguous(), nturn=self.nturn, inplace=True)
        return r.ret, r.flips, r.legal_next

    def step_strings(self, hands):
        """Edax move strings per game ('d3', 'PS', ...), parsed on the host as put_s does."""
        codes = torch.tensor([codec.move_code(h) for h in hands], dtype=torch.uint8)
        return self.step(codes.to(self.device))

    # reference: is_game_over + n_black/n_white result rule (game_runner.py:162, 194-199)
    def result(self):
        """dict(n_black, n_white, diff, terminal, winner) with winner 1 Black, 2 White, 0 draw."""
        r = ops.result(self.boards)
        d = r.diff
        winner = torch.where(d > 0, 1, torch.where(d < 0, 2, 0)).to(torch.uint8)
        return dict(n_black=r.n_black, n_white=r.n_white, diff=d, terminal=r.terminal.bool(), winner=winner)

    def is_game_over(self):
        return ops.result(self.boards).terminal.bool()

    def books(self):
        """Book text (serialize_str, board.py:214-221) of every game: oth_book_text
        on the device, one 67-byte line per game, decoded on the host."""
        raw = ops.book_text(self.boards, self.turn).cpu().numpy().tobytes()
        return raw.decode("ascii").splitlines()
