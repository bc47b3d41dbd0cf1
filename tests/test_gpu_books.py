"""§8f rows on the GPU: book emitter (replay + serialize_str text) and learner
features, against board.py / reference-learner fixtures and the oracle."""
import numpy as np
import pytest
import torch

import oracle
from golden_io import load_json, load_npz

pytestmark = pytest.mark.gpu

from subproc_amd import ops  # noqa: E402
from subproc_amd.books import GameBooks  # noqa: E402

U = ops.to_numpy_u64


def _src(name):
    z = load_npz(name + ".npz")
    start = ops.from_numpy_u64(np.stack([z["start_black"], z["start_white"]], 1), "cuda")
    return z, start, torch.as_tensor(z["start_turn"]).cuda()


def test_books_match_reference_recorder():
    srcs = {n: _src(n) for n in ("rollout_random", "rollout_random_from_mid")}
    gb = {n: GameBooks(torch.as_tensor(z["moves"]).cuda(), torch.as_tensor(z["plies"]).cuda(), st, stt)
          for n, (z, st, stt) in srcs.items()}
    for bk in load_json("books.json"):
        b, g = gb[bk["source"]], bk["game"]
        assert b.lines(g) == bk["lines"]
        recs = b.records(g)
        assert recs == [{"book": r["book"], "whosturn": r["whosturn"], "turn": r["turn"], "end": r["end"]}
                        for r in bk["records"]]
        flat = b.flat_file_bytes(g, "A", "B").decode()
        assert flat == "% Black: A\n% White: B\n" + "".join(line + "\n" for line in bk["lines"])
        for side, col in ((1, 0), (2, 1)):
            f = b.features(side)[g, :len(bk["lines"])].cpu().numpy()
            assert f.tolist() == [c[col] for c in bk["counts"]], (bk["game"], side)


def test_replay_and_text_at_scale_vs_oracle(tmp_path):
    n = 4096
    r = ops.rollout(n, 31, 7, record_moves=True, device="cuda")
    gb = GameBooks.from_rollout(r)
    o = oracle.replay(r.moves.cpu().numpy(), r.plies.cpu().numpy())
    pl = r.plies.cpu().numpy()
    gpu_b = U(gb.pos.boards)
    for g in range(0, n, 97):
        k = int(pl[g]) + 1
        np.testing.assert_array_equal(gpu_b[g, :k], o["boards"][g, :k])
        np.testing.assert_array_equal(gb.pos.turn[g, :k].cpu().numpy(), o["turn"][g, :k])
        np.testing.assert_array_equal(gb.pos.end[g, :k].cpu().numpy(), o["end"][g, :k])
        assert gb.lines(g) == [oracle.serialize_str(b, w, t) for (b, w), t in zip(o["boards"][g, :k], o["turn"][g, :k])]
        assert gb.pos.end[g, k - 1].item() == 1 and gb.pos.end[g, :k - 1].sum().item() == 0
    # final replayed position == rollout final board
    last = gpu_b[np.arange(n), pl.astype(np.int64)]
    np.testing.assert_array_equal(last, U(r.final_boards))
    paths = gb.write_flat_files(str(tmp_path), "t", games=[0, 1])
    assert open(paths[1], "rb").read() == gb.flat_file_bytes(1, "gpu_black", "gpu_white")


def test_features_vs_oracle_random_boards():
    rng = np.random.default_rng(9)
    n = 20000
    occ = rng.integers(0, 2**64, n, dtype=np.uint64) | rng.integers(0, 2**64, n, dtype=np.uint64)
    col = rng.integers(0, 2**64, n, dtype=np.uint64)
    nb = np.stack([occ & col, occ & ~col], 1)
    side = rng.integers(1, 3, n).astype(np.uint8)
    f = ops.features(ops.from_numpy_u64(nb, "cuda"), torch.as_tensor(side).cuda()).cpu().numpy()
    np.testing.assert_array_equal(f, oracle.features(nb, side))


def test_book_text_tail_lengths():
    """Text sizes that are not multiples of 16 bytes (the kernel's partial tail)."""
    for n in (1, 2, 3, 5, 17):
        b, t, _ = ops.reset(n, "cuda")
        txt = ops.book_text(b, t).cpu().numpy().tobytes().decode()
        assert txt == "---------------------------XO------OX--------------------------- O\n" * n


@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 257, 1000])
def test_book_text_random_boards_every_side(n):
    """Arbitrary boards (any occupancy) and side codes 0..3 at ragged sizes --
    lines that share dwords with their neighbours in the kernel's LDS
    assembly, and waves with fewer than 64 lines -- against the host codec."""
    from subproc_amd import codec
    rng = np.random.default_rng(n)
    occ = rng.integers(0, 2**64, n, dtype=np.uint64)
    col = rng.integers(0, 2**64, n, dtype=np.uint64)
    nb = np.stack([occ & col, occ & ~col], 1)
    side = rng.integers(0, 4, n).astype(np.uint8)
    txt = ops.book_text(ops.from_numpy_u64(nb, "cuda"), torch.as_tensor(side).cuda()).cpu().numpy().tobytes().decode()
    want = "".join(codec.serialize_str(int(b), int(w), int(t)) + "\n" for (b, w), t in zip(nb, side))
    assert txt == want


def test_book_text_and_features_unaligned_outputs():
    """Outputs that are not 16-byte aligned (a caller's buffer + 1): the kernels
    assemble each wave's bytes in LDS and fall back to byte stores; the bytes
    equal the aligned call's."""
    from subproc_amd import _lib
    n = 300
    rng = np.random.default_rng(5)
    occ = rng.integers(0, 2**64, n, dtype=np.uint64)
    col = rng.integers(0, 2**64, n, dtype=np.uint64)
    nb = np.stack([occ & col, occ & ~col], 1)
    side = torch.as_tensor(rng.integers(0, 4, n).astype(np.uint8)).cuda()
    b = ops.from_numpy_u64(nb, "cuda")
    L = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    want_txt = ops.book_text(b, side)
    buf = torch.zeros(n * 67 + 32, dtype=torch.uint8, device="cuda")
    assert L.oth_book_text(b.data_ptr(), side.data_ptr(), n, buf.data_ptr() + 1, st) == 0
    assert torch.equal(buf[1:1 + n * 67], want_txt) and int(buf[0]) == 0 and int(buf[1 + n * 67]) == 0
    fs = torch.clamp(side, 1, 2)
    want_f = ops.features(b, fs).reshape(-1)
    buf = torch.zeros(n * 10 + 32, dtype=torch.uint8, device="cuda")
    assert L.oth_features(b.data_ptr(), fs.data_ptr(), buf.data_ptr() + 3, n, st) == 0
    assert torch.equal(buf[3:3 + n * 10], want_f) and int(buf[3 + n * 10]) == 0


def test_replay_full_size_properties():
    """262,144 games (the TD batch and the book-emitter bench size) replayed
    in one launch: every row of every game's stride checked by size-independent
    properties on the device (rows past plies 0; the last recorded position is
    the rollout's final board and the only one with is_game_over; the side to
    move at row p+1 is the one put_s left), and a strided sample of games --
    the last ones included -- against the oracle's mailbox replay."""
    n = 1 << 18
    r = ops.rollout(n, 77, 1 << 30, record_moves=True, device="cuda")
    pos = ops.replay(r.moves, r.plies)
    pl = r.plies.long()
    rows = torch.arange(129, device="cuda")[None, :]
    inside = rows <= pl[:, None]
    assert bool((pos.boards[~inside] == 0).all()) and bool((pos.turn[~inside] == 0).all())
    assert bool((pos.end[~inside] == 0).all())
    last = pos.boards[torch.arange(n, device="cuda"), pl]
    assert torch.equal(last, r.final_boards)
    ends = pos.end.long().sum(1)
    assert bool((ends == 1).all()) and bool((pos.end[torch.arange(n, device="cuda"), pl] == 1).all())
    assert bool(((pos.turn == 1) | (pos.turn == 2))[inside].all())
    idx = np.unique(np.concatenate([np.arange(0, n, 1021), np.arange(n - 64, n)]))
    o = oracle.replay(r.moves.cpu().numpy()[idx], r.plies.cpu().numpy()[idx])
    np.testing.assert_array_equal(U(pos.boards[idx].reshape(-1, 2)).reshape(len(idx), 129, 2), o["boards"])
    np.testing.assert_array_equal(pos.turn[idx].cpu().numpy(), o["turn"])
    np.testing.assert_array_equal(pos.end[idx].cpu().numpy(), o["end"])
