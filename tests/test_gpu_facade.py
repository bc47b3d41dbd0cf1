"""The drop-in Board facade and VecEnv on the GPU, against board.py fixtures."""
import numpy as np
import pytest
import torch

from golden_io import h, load_json, load_npz

pytestmark = pytest.mark.gpu

from subproc_amd import board as gboard  # noqa: E402
from subproc_amd import codec, ops  # noqa: E402
from subproc_amd.env import VecEnv  # noqa: E402


def test_board_opening_strings():
    op = load_json("opening.json")
    b0 = gboard.Board()
    assert str(b0) == op["str"]
    assert b0.is_game_over() == op["is_game_over"]
    assert b0.puttables(1) == [(3, 2), (2, 3), (5, 4), (4, 5)]
    for rec in op["strings"]:
        b = gboard.Board()
        assert b.put_s(rec["s"]) == rec["ret"], rec["s"]
        assert b.bitboards() == (int(rec["black"], 16), int(rec["white"], 16)), rec["s"]
        assert b.turn == rec["turn"] and b.nturn == rec["nturn"]
    for rec in op["index_error"]:
        b = gboard.Board()
        if rec["raises"]:
            with pytest.raises(IndexError):
                b.put_s(rec["s"])


def test_board_replays_golden_games():
    z = load_npz("rollout_random.npz")
    for g in range(0, 256, 16):
        b = gboard.Board()
        for code in z["moves"][g]:
            if code == 255:
                break
            assert not b.is_game_over()
            assert b.put_s(codec.move_str(int(code))) >= 0
        assert b.is_game_over()
        assert b.bitboards() == (int(z["final_black"][g]), int(z["final_white"][g]))
        assert b.n_black() - b.n_white() == int(z["diff"][g])
        assert b.n_empty() == 64 - b.n_black() - b.n_white()


def test_board_edges_and_helpers():
    for e in load_json("edges.json"):
        b = gboard.Board()
        b.deserialize(e["serialize_str"][:64], e["serialize_str"][65], 0)
        assert b.serialize_str() == e["serialize_str"]
        assert b.is_game_over() == e["is_game_over"], e["name"]
        assert b.n_black() == e["n_black"] and b.n_white() == e["n_white"] and b.n_empty() == e["n_empty"]
        lb = sum(1 << (x + 8 * y) for x, y in b.puttables(1))
        assert lb == int(e["legal_black"], 16)
        assert b.n_puttable_for(2) == bin(int(e["legal_white"], 16)).count("1")
    b = gboard.Board()
    assert b.put(1, 3, 2) == 1 and b.turn == 1  # put does not toggle the turn
    b = gboard.Board()
    assert b.hands_for_direc(gboard.D, 1, 3, 2) == [(1, 3, 3)]
    assert b.hands_for_direc(gboard.U, 1, 3, 2) == []
    assert b.is_puttable_at(1, 3, 2) and not b.is_puttable_at(1, 0, 0)
    assert b.mask_count(1, 0xFFFFFFFFFFFFFFFF) == 2 and b.mask_count(0, 0xFFFFFFFFFFFFFFFF) == 60


def test_vecenv_random_games_match_fixture():
    z = load_npz("rollout_random.npz")
    n = len(z["plies"])
    env = VecEnv(n)
    for ply in range(128):
        col = z["moves"][:, ply]
        live = col != 255
        if not live.any():
            break
        moves = torch.as_tensor(np.where(live, col, 64).astype(np.uint8)).cuda()
        legal = ops.to_numpy_u64(env.legal_moves())
        for i in np.nonzero(live)[0][:8]:
            c = int(col[i])
            assert (c == 64 and legal[i] == 0) or (c < 64 and legal[i] >> np.uint64(c) & np.uint64(1))
        # finished games are stepped with a pass, then rolled back by reset_mask-free bookkeeping
        before = env.boards.clone(), env.turn.clone(), env.nturn.clone()
        ret, _, _ = env.step(moves)
        keep = torch.as_tensor(~live).cuda()
        env.boards = torch.where(keep[:, None], before[0], env.boards)
        env.turn = torch.where(keep, before[1], env.turn)
        env.nturn = torch.where(keep, before[2], env.nturn)
        assert (ret.cpu().numpy()[live] >= 0).all()
    res = env.result()
    assert bool(res["terminal"].all())
    fb = ops.to_numpy_u64(env.boards)
    np.testing.assert_array_equal(fb[:, 0], z["final_black"])
    np.testing.assert_array_equal(fb[:, 1], z["final_white"])
    np.testing.assert_array_equal(env.nturn.cpu().numpy(), z["plies"])
    np.testing.assert_array_equal(res["diff"].cpu().numpy(), z["diff"])
    books = env.books()
    assert all(len(s) == 66 for s in books)
    # the device text equals the host codec (pinned to board.py by tests/test_codec.py)
    from subproc_amd import codec
    host = [b + " " + codec.string_from_turn(t)
            for b, t in zip(codec.serialize_boards(ops.to_numpy_u64(env.boards)), env.turn.cpu().tolist())]
    assert books == host


def test_vecenv_strings():
    op = load_json("opening.json")
    env = VecEnv(4)
    ret, flips, _ = env.step_strings(["d3", "C4", "Bf5", "ps"])
    assert ret.cpu().tolist() == [1, 1, 1, 0]
    assert ops.to_numpy_u64(env.boards)[0, 0] == h(op["moves"][0]["black"])
