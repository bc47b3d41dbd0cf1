"""The HIP C-ABI on board.py's answers beyond Black/White play, bit-exact:
oth_legal / oth_step / oth_replay with the side to move Empty or a value no
square holds, and oth_hands from any origin along any direction, against the
fixtures gen_golden.py made from the real board.py (board_api.npz,
side_steps.npz) and against the oracle on random inputs."""
import numpy as np
import pytest
import torch

import oracle
from golden_io import load_npz
from test_board_api import _hands_items, own_hostile

pytestmark = pytest.mark.gpu

from subproc_amd import ops  # noqa: E402

DEV = "cuda"
U = ops.to_numpy_u64


def T(a, dtype=torch.uint8):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dtype).to(DEV)


def B(black, white):
    return ops.from_numpy_u64(np.stack([np.asarray(black, np.uint64), np.asarray(white, np.uint64)], 1), DEV)


def test_side_empty_and_other_every_code():
    z = load_npz("side_steps.npz")
    n = len(z["black"])
    boards, turn = B(z["black"], z["white"]), T(z["turn"])
    np.testing.assert_array_equal(U(ops.legal(boards, turn)), z["legal"])
    for code in range(65):
        nturn = torch.full((n,), 7, dtype=torch.uint8, device=DEV)
        r = ops.step(boards, turn, T(np.full(n, code)), nturn=nturn)
        np.testing.assert_array_equal(r.ret.cpu().numpy(), z["ret"][:, code])
        np.testing.assert_array_equal(U(r.boards)[:, 0], z["next_black"][:, code])
        np.testing.assert_array_equal(U(r.boards)[:, 1], z["next_white"][:, code])
        np.testing.assert_array_equal(r.turn.cpu().numpy(), z["next_turn"][:, code])
        np.testing.assert_array_equal(nturn.cpu().numpy(), z["next_nturn"][:, code])
        np.testing.assert_array_equal(U(r.legal_next), z["next_legal"][:, code])
        changed = (z["black"] ^ z["next_black"][:, code]) | (z["white"] ^ z["next_white"][:, code])
        origin = np.uint64(1 << code) if code < 64 else np.uint64(0)
        np.testing.assert_array_equal(U(r.flips), changed & ~origin)


def test_every_turn_value_random_boards_vs_oracle():
    """Turn bytes 0..255 on random boards, every code 0..66: the oracle (board.py's
    algorithm for any piece value) and the kernel agree, including the fast path
    for 1/2 sitting next to the general one in the same waves."""
    rng = np.random.default_rng(5)
    m = 1 << 16
    occ = rng.integers(0, 2**64, m, dtype=np.uint64) & rng.integers(0, 2**64, m, dtype=np.uint64)
    col = rng.integers(0, 2**64, m, dtype=np.uint64)
    nb = np.stack([occ & col, occ & ~col], 1)
    tt = rng.integers(0, 256, m).astype(np.uint8)
    tt = np.where(rng.random(m) < 0.6, rng.integers(0, 3, m), tt).astype(np.uint8)
    mv = rng.integers(0, 67, m).astype(np.uint8)
    r = ops.step(B(nb[:, 0], nb[:, 1]), T(tt), T(mv))
    o = oracle.step(nb, tt, mv)
    for k in ("boards", "flips", "legal_next"):
        np.testing.assert_array_equal(U(getattr(r, k)), o[k], err_msg=k)
    np.testing.assert_array_equal(r.ret.cpu().numpy(), o["ret"])
    np.testing.assert_array_equal(r.turn.cpu().numpy(), o["turn"])
    np.testing.assert_array_equal(U(ops.legal(B(nb[:, 0], nb[:, 1]), T(tt))), oracle.legal(nb, tt))


def test_hands_fixture_any_origin_any_direction():
    it = _hands_items()
    own, hos = own_hostile(API_BLACK()[it["board"]], API_WHITE()[it["board"]], it["piece"])
    cols = [torch.as_tensor(np.ascontiguousarray(it[k], np.int64)).to(DEV) for k in ("x", "y", "dx", "dy")]
    got = ops.hands(ops.from_numpy_u64(own, DEV), ops.from_numpy_u64(hos, DEV), *cols)
    np.testing.assert_array_equal(got.cpu().numpy(), it["want"])


def test_hands_random_vs_oracle_and_extreme_coordinates():
    rng = np.random.default_rng(9)
    m = 1 << 15
    occ = rng.integers(0, 2**64, m, dtype=np.uint64) | rng.integers(0, 2**64, m, dtype=np.uint64)
    col = rng.integers(0, 2**64, m, dtype=np.uint64)
    nb = np.stack([occ & col, occ & ~col], 1)
    piece = rng.integers(0, 4, m).astype(np.uint8)
    big = np.array([-(1 << 63), (1 << 63) - 1, -(1 << 62), 1 << 40], np.int64)
    x = np.where(rng.random(m) < 0.05, rng.choice(big, m), rng.integers(-3, 11, m)).astype(np.int64)
    y = np.where(rng.random(m) < 0.05, rng.choice(big, m), rng.integers(-3, 11, m)).astype(np.int64)
    dx = np.where(rng.random(m) < 0.05, rng.choice(big, m), rng.integers(-2, 3, m)).astype(np.int64)
    dy = rng.integers(-2, 3, m).astype(np.int64)
    want = oracle.hands(nb, piece, x, y, dx, dy)
    own, hos = own_hostile(nb[:, 0], nb[:, 1], piece)
    cols = [torch.as_tensor(v).to(DEV) for v in (x, y, dx, dy)]
    got = ops.hands(ops.from_numpy_u64(own, DEV), ops.from_numpy_u64(hos, DEV), *cols)
    np.testing.assert_array_equal(got.cpu().numpy(), want)


def test_replay_from_side_empty_starts_vs_oracle():
    """oth_replay's put_s for any side to move: starts with Empty or no-colour
    turns, random move codes (legal or not), against the oracle's replay."""
    rng = np.random.default_rng(3)
    n = 2048
    pos = ops.sample_midgame(n, 17, device=DEV)
    st = np.where(rng.random(n) < 0.5, 0, rng.integers(0, 5, n)).astype(np.uint8)
    st[::7] = rng.choice([126, 127, 128, 200, 255], len(st[::7]))  # turns the kernel stages as an escape
    moves = rng.integers(0, 66, (n, 128)).astype(np.uint8)
    plies = rng.integers(0, 129, n).astype(np.uint8)
    r = ops.replay(T(moves), T(plies), start=pos.boards, start_turn=T(st))
    o = oracle.replay(moves, plies, start=U(pos.boards), start_turn=st)
    np.testing.assert_array_equal(U(r.boards), o["boards"])
    np.testing.assert_array_equal(r.turn.cpu().numpy(), o["turn"])
    np.testing.assert_array_equal(r.end.cpu().numpy(), o["end"])


def API_BLACK():
    return load_npz("board_api.npz")["black"]


def API_WHITE():
    return load_npz("board_api.npz")["white"]


@pytest.mark.parametrize("n", [1, 255, 257, 1000])
def test_replay_unaligned_buffers_and_ragged_blocks_vs_oracle(n):
    """oth_replay with move records and turn/end outputs that are not 16-B
    aligned (the kernel's byte paths), block-ragged n, start turns >= 127, and
    outputs pre-filled with garbage: rows past plies read back as 0."""
    from subproc_amd import _lib

    rng = np.random.default_rng(n)
    pos = ops.sample_midgame(n, 23, device=DEV)
    st = rng.choice([0, 1, 2, 3, 127, 255], n).astype(np.uint8)
    moves = rng.integers(0, 66, (n, 128)).astype(np.uint8)
    moves[rng.random((n, 128)) < 0.5] = 64  # plenty of passes: turns toggle early
    plies = rng.integers(0, 129, n).astype(np.uint8)
    o = oracle.replay(moves, plies, start=U(pos.boards), start_turn=st)
    for off in (0, 1, 3):
        mv = torch.zeros(n * 128 + off, dtype=torch.uint8, device=DEV)
        mv[off:] = T(moves.reshape(-1))
        pb = torch.zeros((n, 129, 2), dtype=torch.int64, device=DEV)
        pt = torch.full((n * 129 + off,), 0xAB, dtype=torch.uint8, device=DEV)
        pe = torch.full((n * 129 + off,), 0xCD, dtype=torch.uint8, device=DEV)
        stt, pl = T(st), T(plies)
        rc = _lib.load().oth_replay(pos.boards.data_ptr(), stt.data_ptr(), mv.data_ptr() + off, pl.data_ptr(),
                                    pb.data_ptr(), pt.data_ptr() + off, pe.data_ptr() + off, n,
                                    torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        np.testing.assert_array_equal(U(pb), o["boards"], err_msg=f"off {off}")
        np.testing.assert_array_equal(pt[off:].cpu().numpy().reshape(n, 129), o["turn"], err_msg=f"off {off}")
        np.testing.assert_array_equal(pe[off:].cpu().numpy().reshape(n, 129), o["end"], err_msg=f"off {off}")
        assert (pt[:off].cpu().numpy() == 0xAB).all() and (pe[:off].cpu().numpy() == 0xCD).all()
