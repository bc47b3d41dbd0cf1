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
            f = b.features(side)[b.game_rows(g)].cpu().numpy()
            assert f.tolist() == [c[col] for c in bk["counts"]], (bk["game"], side)


def test_replay_and_text_at_scale_vs_oracle(tmp_path):
    n = 4096
    r = ops.rollout(n, 31, 7, record_moves=True, device="cuda")
    gb = GameBooks.from_rollout(r)
    o = oracle.replay(r.moves.cpu().numpy(), r.plies.cpu().numpy())
    pl = r.plies.cpu().numpy()
    gpu_b = U(gb.pos.boards)
    off = gb.pos.row_off.cpu().numpy()
    for g in range(0, n, 97):
        k = int(pl[g]) + 1
        rows = gb.game_rows(g)
        np.testing.assert_array_equal(gpu_b[rows], o["boards"][g, :k])
        np.testing.assert_array_equal(gb.pos.turn[rows].cpu().numpy(), o["turn"][g, :k])
        np.testing.assert_array_equal(gb.pos.end[rows].cpu().numpy(), o["end"][g, :k])
        assert gb.lines(g) == [oracle.serialize_str(b, w, t) for (b, w), t in zip(o["boards"][g, :k], o["turn"][g, :k])]
        assert int(gb.pos.end[rows][-1]) == 1 and int(gb.pos.end[rows][:-1].sum()) == 0
    # final replayed position == rollout final board
    last = gpu_b[off + pl.astype(np.int64)]
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


def test_replay_rows_equals_the_strided_table():
    """oth_replay_rows writes each game's rows 0..plies at row_off[g]: the same
    rows as oth_replay's stride, from the opening and from mid-game starts
    (random policy and greedy, whose game lengths differ), 262,144 games."""
    for n, kw in ((1 << 18, {}), (4096, {"policy": "greedy"})):
        r = ops.rollout(n, 5, 1 << 33, record_moves=True, device="cuda", **kw)
        full = ops.replay(r.moves, r.plies)
        pk = ops.replay_rows(r.moves, r.plies)
        pl = r.plies.long()
        inside = torch.arange(129, device="cuda")[None, :] <= pl[:, None]
        assert pk.boards.shape[0] == int(inside.sum())
        assert torch.equal(pk.boards, full.boards[inside])
        assert torch.equal(pk.turn, full.turn[inside]) and torch.equal(pk.end, full.end[inside])
    z, st, stt = _src("rollout_random_from_mid")
    mv, plz = torch.as_tensor(z["moves"]).cuda(), torch.as_tensor(z["plies"]).cuda()
    full = ops.replay(mv, plz, st, stt)
    pk = ops.replay_rows(mv, plz, st, stt)
    inside = torch.arange(129, device="cuda")[None, :] <= plz.long()[:, None]
    assert torch.equal(pk.boards, full.boards[inside]) and torch.equal(pk.turn, full.turn[inside])
    assert torch.equal(pk.end, full.end[inside])


def test_replay_rows_odd_offsets_and_outputs():
    """Row offsets that are not the prefix sum (a gap after every game, so a
    block's turn/end range overruns its LDS stage and it stores them directly),
    outputs at +1 byte (not 16-B aligned), and start turns 0 and 200 (the
    staged escape): every game's rows equal the strided table's, and the
    bytes between games are left as they were."""
    from subproc_amd import _lib
    n = 700
    r = ops.rollout(n, 3, 0, record_moves=True, device="cuda")
    rng = np.random.default_rng(4)
    start = r.final_boards.clone()
    stt = torch.as_tensor(rng.choice([0, 1, 2, 200], n).astype(np.uint8)).cuda()
    mv = torch.as_tensor(rng.integers(0, 66, (n, 128)).astype(np.uint8)).cuda()
    mv[:, 0] = 64  # a pass first: the start turn row, then put_s turns
    pl = torch.as_tensor(rng.integers(0, 129, n).astype(np.uint8)).cuda()
    full = ops.replay(mv, pl, start, stt)
    inside = torch.arange(129, device="cuda")[None, :] <= pl.long()[:, None]
    L = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    for gap in (0, 200):
        cnt = pl.long() + 1 + gap
        off = (torch.cumsum(cnt, 0) - cnt).contiguous()
        total = int(cnt.sum())
        b = torch.full((total + 1, 2), 7, dtype=torch.int64, device="cuda")
        t = torch.full((total + 17,), 0xAB, dtype=torch.uint8, device="cuda")
        e = torch.full((total + 17,), 0xCD, dtype=torch.uint8, device="cuda")
        assert L.oth_replay_rows(start.data_ptr(), stt.data_ptr(), mv.data_ptr(), pl.data_ptr(), off.data_ptr(),
                                 b.data_ptr(), t.data_ptr() + 1, e.data_ptr() + 1, n, s) == 0
        rows = (off[:, None] + torch.arange(129, device="cuda")[None, :])[inside]
        assert torch.equal(b[rows], full.boards[inside]), gap
        assert torch.equal(t[1:][rows], full.turn[inside]) and torch.equal(e[1:][rows], full.end[inside]), gap
        untouched = torch.ones(total, dtype=torch.bool, device="cuda")
        untouched[rows] = False
        assert bool((t[1:1 + total][untouched] == 0xAB).all()) and bool((e[1:1 + total][untouched] == 0xCD).all())
        assert int(t[0]) == 0xAB and bool((t[1 + total:] == 0xAB).all())


def test_replay_rows_non_monotonic_offsets():
    """Row offsets that are not increasing: games laid out in
    reverse order, shuffled inside each 256-game block (the block's rows still
    one range: staged), and shuffled over the whole launch (ranges overrun the
    stage: direct).  The stage range is taken over every game of a block, so
    every game's rows equal the strided table's, with aligned and +1 outputs."""
    from subproc_amd import _lib
    n = 1500
    r = ops.rollout(n, 11, 77, record_moves=True, device="cuda")
    full = ops.replay(r.moves, r.plies)
    pl = r.plies.long()
    inside = torch.arange(129, device="cuda")[None, :] <= pl[:, None]
    cnt = (pl + 1).cpu().numpy()
    rng = np.random.default_rng(9)
    within = np.concatenate([rng.permutation(np.arange(b, min(b + 256, n))) for b in range(0, n, 256)])
    L = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    total = int(cnt.sum())
    for order in (np.arange(n)[::-1], within, rng.permutation(n)):
        # game order[k] is the k-th in memory: disjoint rows, offsets out of order
        off_np = np.zeros(n, np.int64)
        off_np[order] = np.cumsum(cnt[order]) - cnt[order]
        off = torch.as_tensor(off_np).cuda()
        for shift in (0, 1):
            b = torch.full((total, 2), 7, dtype=torch.int64, device="cuda")
            t = torch.full((total + 1,), 0xAB, dtype=torch.uint8, device="cuda")
            e = torch.full((total + 1,), 0xCD, dtype=torch.uint8, device="cuda")
            assert L.oth_replay_rows(None, None, r.moves.data_ptr(), r.plies.data_ptr(), off.data_ptr(),
                                     b.data_ptr(), t.data_ptr() + shift, e.data_ptr() + shift, n, s) == 0
            rows = (off[:, None] + torch.arange(129, device="cuda")[None, :])[inside]
            assert torch.equal(b[rows], full.boards[inside])
            tt, ee = t[shift:shift + total], e[shift:shift + total]
            assert torch.equal(tt[rows], full.turn[inside]) and torch.equal(ee[rows], full.end[inside])


def test_replay_rows_non_monotonic_offsets_escaped_turns():
    """Offsets shuffled inside each 256-game block (staged) with start turns
    0, 1, 2, 200 and a pass first, so escaped turn bytes (start turn >= 127)
    sit in blocks whose offsets do not increase: the escape's
    game is found by a scan of the block's rows, not a binary search."""
    from subproc_amd import _lib
    n = 1500
    rng = np.random.default_rng(21)
    r = ops.rollout(n, 13, 5, record_moves=True, device="cuda")
    start = r.final_boards.clone()
    stt = torch.as_tensor(rng.choice([0, 1, 2, 200], n).astype(np.uint8)).cuda()
    mv = torch.as_tensor(rng.integers(0, 66, (n, 128)).astype(np.uint8)).cuda()
    mv[:, 0] = 64  # a pass first: row 0 holds the start turn (escaped when 200), then put_s turns
    pl = torch.as_tensor(rng.integers(0, 40, n).astype(np.uint8)).cuda()
    full = ops.replay(mv, pl, start, stt)
    inside = torch.arange(129, device="cuda")[None, :] <= pl.long()[:, None]
    cnt = (pl.long() + 1).cpu().numpy()
    within = np.concatenate([rng.permutation(np.arange(b, min(b + 256, n))) for b in range(0, n, 256)])
    L = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    total = int(cnt.sum())
    for order in (np.arange(n)[::-1], within):
        off_np = np.zeros(n, np.int64)
        off_np[order] = np.cumsum(cnt[order]) - cnt[order]
        off = torch.as_tensor(off_np).cuda()
        for shift in (0, 1):
            b = torch.full((total, 2), 7, dtype=torch.int64, device="cuda")
            t = torch.full((total + 1,), 0xAB, dtype=torch.uint8, device="cuda")
            e = torch.full((total + 1,), 0xCD, dtype=torch.uint8, device="cuda")
            assert L.oth_replay_rows(start.data_ptr(), stt.data_ptr(), mv.data_ptr(), pl.data_ptr(), off.data_ptr(),
                                     b.data_ptr(), t.data_ptr() + shift, e.data_ptr() + shift, n, s) == 0
            rows = (off[:, None] + torch.arange(129, device="cuda")[None, :])[inside]
            assert torch.equal(b[rows], full.boards[inside])
            tt, ee = t[shift:shift + total], e[shift:shift + total]
            assert int((full.turn[inside] == 200).sum()) > 100  # escapes are exercised
            assert torch.equal(tt[rows], full.turn[inside]) and torch.equal(ee[rows], full.end[inside])
