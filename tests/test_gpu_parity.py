"""GPU parity: the HIP kernels (through the C-ABI, via subproc_amd.ops) against the
golden fixtures from the real board.py and against the C oracle at scale.
Bit-exact everywhere (integer/bitwise work)."""
import numpy as np
import pytest
import torch

import oracle
from golden_io import ROLLOUT_FIXTURES, h, load_json, load_npz

pytestmark = pytest.mark.gpu

from subproc_amd import ops  # noqa: E402

DEV = "cuda"
U = ops.to_numpy_u64


def T(a, dtype=torch.uint8):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dtype).to(DEV)


def B(black, white):
    return ops.from_numpy_u64(np.stack([np.asarray(black, np.uint64), np.asarray(white, np.uint64)], 1), DEV)


def test_reset():
    op = load_json("opening.json")
    b, t, nt = ops.reset(1000, DEV)
    b = U(b)
    assert (b[:, 0] == h(op["black"])).all() and (b[:, 1] == h(op["white"])).all()
    assert (t.cpu() == 1).all() and (nt.cpu() == 0).all()


def test_opening_known_answers():
    op = load_json("opening.json")
    boards = B([h(op["black"])] * 2, [h(op["white"])] * 2)
    leg = U(ops.legal(boards, T([1, 2])))
    assert leg[0] == h(op["legal_black"]) and leg[1] == h(op["legal_white"])
    ms = op["moves"]
    n = len(ms)
    boards = B([h(op["black"])] * n, [h(op["white"])] * n)
    nturn = torch.zeros(n, dtype=torch.uint8, device=DEV)
    r = ops.step(boards, T([op["turn"]] * n), T([m["sq"] for m in ms]), nturn=nturn)
    for i, m in enumerate(ms):
        assert int(r.ret[i]) == m["ret"]
        assert U(r.flips)[i] == h(m["flips"])
        assert U(r.boards)[i, 0] == h(m["black"]) and U(r.boards)[i, 1] == h(m["white"])
        assert int(r.turn[i]) == m["turn"] and int(nturn[i]) == m["nturn"]


def test_midgame_every_code():
    z = load_npz("midgame_step.npz")
    n = len(z["black"])
    boards = B(z["black"], z["white"])
    turn = T(z["turn"])
    assert (U(ops.legal(boards, turn)) == z["legal"]).all()
    for code in range(65):
        nturn = torch.zeros(n, dtype=torch.uint8, device=DEV)
        r = ops.step(boards, turn, T(np.full(n, code)), nturn=nturn)
        np.testing.assert_array_equal(r.ret.cpu().numpy(), z["ret"][:, code])
        np.testing.assert_array_equal(U(r.boards)[:, 0], z["next_black"][:, code])
        np.testing.assert_array_equal(U(r.boards)[:, 1], z["next_white"][:, code])
        np.testing.assert_array_equal(r.turn.cpu().numpy(), z["next_turn"][:, code])
        np.testing.assert_array_equal(nturn.cpu().numpy(), z["next_nturn"][:, code])
        np.testing.assert_array_equal(U(r.legal_next), z["next_legal"][:, code])
        # flips = opponent discs that changed colour
        mover_black = z["turn"] == 1
        opp0 = np.where(mover_black, z["white"], z["black"])
        opp1 = np.where(mover_black, z["next_white"][:, code], z["next_black"][:, code])
        np.testing.assert_array_equal(U(r.flips), opp0 & ~opp1)


def test_edges():
    for e in load_json("edges.json"):
        n = len(e["steps"])
        boards = B([h(e["black"])] * n, [h(e["white"])] * n)
        res = ops.result(boards[:1])
        assert int(res.terminal[0]) == int(e["is_game_over"]), e["name"]
        assert int(res.n_black[0]) == e["n_black"] and int(res.n_white[0]) == e["n_white"], e["name"]
        assert int(res.diff[0]) == e["n_black"] - e["n_white"]
        r = ops.step(boards, T([e["turn"]] * n), T([s["code"] for s in e["steps"]]))
        for i, s in enumerate(e["steps"]):
            assert int(r.ret[i]) == s["ret"], (e["name"], s["code"])
            assert U(r.boards)[i, 0] == h(s["black"]) and U(r.boards)[i, 1] == h(s["white"]), (e["name"], s["code"])
            assert int(r.turn[i]) == s["turn"]


def test_invalid_codes_and_odd_turns():
    """Codes > 64 are -1 with the state unchanged.  Side Empty (0) on the
    opening: d3 flanks e4 (a Black run ending on the empty f5), so e4 is
    "flipped" to Empty and the turn goes to Black (board.py:155-209); a side
    no square holds (3) takes only a pass, which also hands over to Black."""
    b, t, _ = ops.reset(8, DEV)
    r = ops.step(b, T([1, 1, 1, 0, 3, 2, 3, 0]), T([65, 200, 255, 19, 19, 64, 64, 0]))
    assert r.ret.cpu().tolist() == [-1, -1, -1, 1, -1, 0, 0, -1]
    assert r.turn.cpu().tolist() == [1, 1, 1, 1, 3, 1, 1, 0]
    bo = U(r.boards)
    assert (bo[[0, 1, 2, 4, 5, 6, 7]] == U(b)[[0, 1, 2, 4, 5, 6, 7]]).all()
    e4 = np.uint64(1 << (4 + 8 * 3))
    assert bo[3, 0] == U(b)[3, 0] & ~e4 and bo[3, 1] == U(b)[3, 1]
    assert U(r.flips)[3] == e4


def test_inplace_step_aliasing():
    z = load_npz("midgame_step.npz")
    boards = B(z["black"], z["white"])
    turn = T(z["turn"])
    lg = U(ops.legal(boards, turn))
    moves = np.array([(int(x) & -int(x)).bit_length() - 1 if x else 64 for x in lg], np.uint8)
    ref = ops.step(boards, turn, T(moves))
    b2, t2 = boards.clone(), turn.clone()
    ops.step(b2, t2, T(moves), inplace=True)
    assert (U(b2) == U(ref.boards)).all() and (t2.cpu() == ref.turn.cpu()).all()


@pytest.mark.parametrize("n,off", [(1, 0), (3, 0), (4, 0), (4093, 0), (4096, 1), (4097, 3), (1023, 2)])
def test_step_ragged_and_unaligned(n, off):
    """Ragged sizes and offset views (byte arrays at odd addresses) against the
    oracle, including the uint8 nturn wrap at 255."""
    rng = np.random.default_rng(n + off)
    m = n + off
    occ = rng.integers(0, 2**64, m, dtype=np.uint64) & rng.integers(0, 2**64, m, dtype=np.uint64)
    col = rng.integers(0, 2**64, m, dtype=np.uint64)
    nb = np.stack([occ & col, occ & ~col], 1)
    tt = rng.integers(0, 4, m).astype(np.uint8)
    mv = rng.integers(0, 66, m).astype(np.uint8)
    nt0 = rng.choice(np.array([0, 1, 127, 128, 254, 255], np.uint8), m)
    boards, turn, move = B(nb[:, 0], nb[:, 1])[off:], T(tt)[off:], T(mv)[off:]
    nturn = T(nt0)[off:]
    r = ops.step(boards, turn, move, nturn=nturn)
    o = oracle.step(nb[off:], tt[off:], mv[off:])
    assert (U(r.boards) == o["boards"]).all()
    assert (U(r.flips) == o["flips"]).all()
    assert (U(r.legal_next) == o["legal_next"]).all()
    assert (r.ret.cpu().numpy() == o["ret"]).all()
    assert (r.turn.cpu().numpy() == o["turn"]).all()
    want_nt = (nt0[off:].astype(np.int64) + (o["ret"] >= 0)).astype(np.uint8)
    np.testing.assert_array_equal(nturn.cpu().numpy(), want_nt)


def test_zero_and_bad_args():
    e = torch.empty((0, 2), dtype=torch.int64, device=DEV)
    r = ops.step(e, torch.empty(0, dtype=torch.uint8, device=DEV), torch.empty(0, dtype=torch.uint8, device=DEV))
    assert r.ret.numel() == 0
    with pytest.raises(ValueError):
        ops.legal(torch.zeros((4, 2), dtype=torch.int64), torch.zeros(4, dtype=torch.uint8))
    with pytest.raises(TypeError):
        ops.legal(torch.zeros((4, 2), dtype=torch.int32, device=DEV), torch.zeros(4, dtype=torch.uint8, device=DEV))


@pytest.mark.parametrize("name", ROLLOUT_FIXTURES)
def test_rollout_fixtures(name):
    z = load_npz(name + ".npz")
    n = len(z["plies"])
    from_mid = "from_mid" in name
    policy = {0: "random", 1: "greedy", 2: "eval"}[int(z["policy"])]
    r = ops.rollout(n, int(z["seed"]), int(z["game_id0"]), policy, int(z["n_random"]),
                    start=B(z["start_black"], z["start_white"]) if from_mid else None,
                    start_turn=T(z["start_turn"]) if from_mid else None, record_moves=True, device=DEV,
                    weights=z.get("weights"), weights_white=z.get("weights_white"))
    np.testing.assert_array_equal(r.moves.cpu().numpy(), z["moves"])
    np.testing.assert_array_equal(r.plies.cpu().numpy(), z["plies"])
    np.testing.assert_array_equal(r.diff.cpu().numpy(), z["diff"])
    np.testing.assert_array_equal(U(r.final_boards)[:, 0], z["final_black"])
    np.testing.assert_array_equal(U(r.final_boards)[:, 1], z["final_white"])
    hist = r.hist.cpu().numpy()
    np.testing.assert_array_equal(hist[:129], np.bincount(z["diff"].astype(np.int64) + 64, minlength=129))
    assert hist[132] == int(z["plies"].sum().astype(np.int64))


def test_sample_midgame_fixture():
    z = load_npz("sample_midgame.npz")
    n = len(z["move"])
    p = ops.sample_midgame(n, int(z["seed"]), device=DEV)
    np.testing.assert_array_equal(U(p.boards)[:, 0], z["black"])
    np.testing.assert_array_equal(U(p.boards)[:, 1], z["white"])
    np.testing.assert_array_equal(p.turn.cpu().numpy(), z["turn"])
    np.testing.assert_array_equal(p.nturn.cpu().numpy(), z["nturn"])
    np.testing.assert_array_equal(p.move.cpu().numpy(), z["move"])


# --------------------------------------------------------------------------- at scale vs oracle
def test_config2_step_65536_vs_oracle():
    n = 65536
    p = ops.sample_midgame(n, 0x5EED, device=DEV)
    o = oracle.sample_midgame(n, 0x5EED)
    assert (U(p.boards) == o["boards"]).all() and (p.move.cpu().numpy() == o["move"]).all()
    r = ops.step(p.boards, p.turn, p.move)
    ro = oracle.step(o["boards"], o["turn"], o["move"])
    assert (U(r.boards) == ro["boards"]).all()
    assert (U(r.flips) == ro["flips"]).all()
    assert (U(r.legal_next) == ro["legal_next"]).all()
    assert (r.ret.cpu().numpy() == ro["ret"]).all()
    assert (r.turn.cpu().numpy() == ro["turn"]).all()
    assert (r.ret.cpu().numpy() >= 1).all()


def test_every_code_random_boards_vs_oracle():
    """Arbitrary (even unreachable) disjoint boards, every move code, both sides."""
    rng = np.random.default_rng(3)
    n = 8192
    occ = rng.integers(0, 2**64, n, dtype=np.uint64) & rng.integers(0, 2**64, n, dtype=np.uint64)
    col = rng.integers(0, 2**64, n, dtype=np.uint64)
    black, white = occ & col, occ & ~col
    boards = B(black, white)
    nb = np.stack([black, white], 1)
    for turn in (1, 2):
        tt = np.full(n, turn, np.uint8)
        assert (U(ops.legal(boards, T(tt))) == oracle.legal(nb, tt)).all()
        for code in range(0, 65, 3):
            mv = np.full(n, code, np.uint8)
            r = ops.step(boards, T(tt), T(mv))
            o = oracle.step(nb, tt, mv)
            assert (U(r.boards) == o["boards"]).all(), code
            assert (U(r.flips) == o["flips"]).all(), code
            assert (U(r.legal_next) == o["legal_next"]).all(), code
            assert (r.ret.cpu().numpy() == o["ret"]).all(), code
    res = ops.result(boards)
    ores = oracle.result(nb)
    for k in ("n_black", "n_white", "diff", "terminal"):
        assert (getattr(res, k).cpu().numpy() == ores[k]).all(), k


def test_every_code_all_densities_vs_oracle():
    """Every (board, code, side) triple over boards from nearly empty to nearly
    full (runs reaching the edges, long runs, rays blocked by either colour):
    the step's carry-along-the-ray flips and the next mover's legal mask."""
    rng = np.random.default_rng(11)
    per = 1024
    parts = []
    for k in (1, 2, 3, 4, 6):  # occupancy 1 - 2^-k: 50% ... 98%
        occ = np.full(per, ~np.uint64(0), np.uint64)
        for _ in range(k):
            occ &= ~rng.integers(0, 2**64, per, dtype=np.uint64)
        parts.append(~occ)
    occ = np.concatenate(parts + [rng.integers(0, 2**64, per, dtype=np.uint64) & rng.integers(0, 2**64, per,
                                                                                              dtype=np.uint64)])
    col = rng.integers(0, 2**64, len(occ), dtype=np.uint64)
    black, white = occ & col, occ & ~col
    n = len(occ) * 65
    nb = np.repeat(np.stack([black, white], 1), 65, axis=0)
    mv = np.tile(np.arange(65, dtype=np.uint8), len(occ))
    boards = B(nb[:, 0], nb[:, 1])
    for turn in (1, 2):
        tt = np.full(n, turn, np.uint8)
        r = ops.step(boards, T(tt), T(mv))
        o = oracle.step(nb, tt, mv)
        assert (U(r.flips) == o["flips"]).all(), turn
        assert (U(r.boards) == o["boards"]).all(), turn
        assert (U(r.legal_next) == o["legal_next"]).all(), turn
        assert (r.ret.cpu().numpy() == o["ret"]).all(), turn
        assert (r.turn.cpu().numpy() == o["turn"]).all(), turn


def test_mixed_side_codes_every_code_vs_oracle():
    """Every lane its own side code -- Black, White, Empty (board.py's turn
    after deserialize with a side string other than 'O'/'X') and codes no
    square holds -- over boards of every density and every move code: the
    step kernel's any-side path runs beside the fast path inside the same
    waves, and legal/step/next-legal/turn/ret equal the oracle."""
    rng = np.random.default_rng(17)
    per = 512
    parts = []
    for k in (1, 2, 4):
        occ = np.full(per, ~np.uint64(0), np.uint64)
        for _ in range(k):
            occ &= ~rng.integers(0, 2**64, per, dtype=np.uint64)
        parts.append(~occ)
    occ = np.concatenate(parts)
    col = rng.integers(0, 2**64, len(occ), dtype=np.uint64)
    black, white = occ & col, occ & ~col
    n = len(occ) * 65
    nb = np.repeat(np.stack([black, white], 1), 65, axis=0)
    mv = np.tile(np.arange(65, dtype=np.uint8), len(occ))
    tt = rng.choice(np.array([0, 1, 1, 2, 2, 3, 255], np.uint8), n)
    boards = B(nb[:, 0], nb[:, 1])
    assert (U(ops.legal(boards, T(tt))) == oracle.legal(nb, tt)).all()
    r = ops.step(boards, T(tt), T(mv))
    o = oracle.step(nb, tt, mv)
    assert (U(r.flips) == o["flips"]).all()
    assert (U(r.boards) == o["boards"]).all()
    assert (U(r.legal_next) == o["legal_next"]).all()
    assert (r.ret.cpu().numpy() == o["ret"]).all()
    assert (r.turn.cpu().numpy() == o["turn"]).all()


def test_rollout_random_65536_vs_oracle():
    n = 65536
    r = ops.rollout(n, 0x5EED, 0, device=DEV)
    o = oracle.rollout(n, 0x5EED, 0)
    assert (U(r.final_boards) == o["final_boards"]).all()
    assert (r.diff.cpu().numpy() == o["diff"]).all()
    assert (r.plies.cpu().numpy() == o["plies"]).all()
    assert (r.hist.cpu().numpy() == o["hist"]).all()


def test_rollout_greedy_4096_vs_oracle():
    n = 4096
    r = ops.rollout(n, 42, 1 << 20, "greedy", 10, device=DEV)
    o = oracle.rollout(n, 42, 1 << 20, policy=1, n_random=10)
    assert (U(r.final_boards) == o["final_boards"]).all()
    assert (r.plies.cpu().numpy() == o["plies"]).all()
    assert (r.hist.cpu().numpy() == o["hist"]).all()


def test_rollout_eval_4096_vs_oracle():
    from subproc_amd.params import DEFAULT_WEIGHTS
    n = 4096
    for w in (DEFAULT_WEIGHTS, np.random.default_rng(5).integers(-127, 128, (4, 9)).astype(np.int8)):
        r = ops.rollout(n, 43, 1 << 21, "eval", 10, weights=w, device=DEV)
        o = oracle.rollout(n, 43, 1 << 21, policy=2, n_random=10, weights=w)
        assert (U(r.final_boards) == o["final_boards"]).all()
        assert (r.plies.cpu().numpy() == o["plies"]).all()
        assert (r.hist.cpu().numpy() == o["hist"]).all()


def test_eval_values():
    z = load_npz("eval_values.npz")
    boards = B(z["black"], z["white"])
    n = len(z["black"])
    for col, side in ((0, 1), (1, 2), (2, 0)):  # 'O', 'X', '-' (turn_from_string -> Empty)
        sides = T(np.full(n, side))
        np.testing.assert_array_equal(ops.features(boards, sides).cpu().numpy(), z["counts"][:, col])
        for wk, ek in (("weights_default", "eval_default"), ("weights_rand", "eval_rand")):
            got = ops.evaluate(boards, sides, z[wk])
            np.testing.assert_array_equal(got.cpu().numpy(), z[ek][:, col])


def test_eval_random_boards_vs_oracle():
    """Arbitrary disjoint boards (every disc count), all three side codes."""
    rng = np.random.default_rng(9)
    n = 32768
    occ = rng.integers(0, 2**64, n, dtype=np.uint64) & rng.integers(0, 2**64, n, dtype=np.uint64)
    occ[: n // 4] = rng.integers(0, 2**64, n // 4, dtype=np.uint64)  # dense boards
    col = rng.integers(0, 2**64, n, dtype=np.uint64)
    nb = np.stack([occ & col, occ & ~col], 1)
    w = rng.integers(-128, 128, (4, 9)).astype(np.int8)
    side = rng.integers(0, 4, n).astype(np.uint8)
    got = ops.evaluate(B(nb[:, 0], nb[:, 1]), T(side), w).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.evaluate(nb, side, w))
    feats = ops.features(B(nb[:, 0], nb[:, 1]), T(side)).cpu().numpy()
    np.testing.assert_array_equal(feats, oracle.features(nb, side))


def test_rollout_from_start_positions_vs_oracle():
    from subproc_amd.params import DEFAULT_WEIGHTS
    n = 16384
    p = ops.sample_midgame(n, 11, device=DEV)
    for policy, pid in (("random", 0), ("greedy", 1), ("eval", 2)):
        w = DEFAULT_WEIGHTS if pid == 2 else None
        r = ops.rollout(n, 5, 77, policy, 0, start=p.boards, start_turn=p.turn, record_moves=True, device=DEV,
                        weights=w)
        o = oracle.rollout(n, 5, 77, pid, 0, start=U(p.boards), start_turn=p.turn.cpu().numpy(),
                           record_moves=True, weights=w)
        assert (r.moves.cpu().numpy() == o["moves"]).all(), policy
        assert (U(r.final_boards) == o["final_boards"]).all(), policy
        assert (r.hist.cpu().numpy() == o["hist"]).all(), policy


# --------------------------------------------------------------------------- full size: every game
def _oracle_full(res, n, seed, policy, n_random, weights=None):
    """Every game of a full-size launch against the OpenMP oracle
    (oracle.rollout on all host threads: OMP_NUM_THREADS = 16 on the GPU box).
    The rule matched is game_runner.py:165-201 with board.py:192-209."""
    o = oracle.rollout(n, seed, 0, policy=policy, n_random=n_random, weights=weights, n_threads=0)
    np.testing.assert_array_equal(U(res.final_boards), o["final_boards"])
    np.testing.assert_array_equal(res.diff.cpu().numpy(), o["diff"])
    np.testing.assert_array_equal(res.plies.cpu().numpy(), o["plies"])
    np.testing.assert_array_equal(res.hist.cpu().numpy(), o["hist"])


def test_config3_full_size_vs_oracle():
    """batch 1,048,576 random games (config 3): every game's final boards, diff
    and plies and the histogram bit-exact against the oracle, plus determinism,
    split invariance and the terminal / histogram properties.  The oracle's
    1M random games take ~5 s of 16 host threads on the GPU box (the bench's
    cpu_baseline rate, 1.25e7 env-steps/s)."""
    n = 1 << 20
    a = ops.rollout(n, 0x5EED, 0, device=DEV)
    b = ops.rollout(n, 0x5EED, 0, device=DEV)
    assert torch.equal(a.final_boards, b.final_boards) and torch.equal(a.hist, b.hist)
    h1 = ops.rollout(n // 2 + 12345, 0x5EED, 0, device=DEV)
    h2 = ops.rollout(n - (n // 2 + 12345), 0x5EED, n // 2 + 12345, device=DEV)
    assert torch.equal(torch.cat([h1.final_boards, h2.final_boards]), a.final_boards)
    assert torch.equal(h1.hist + h2.hist, a.hist)
    res = ops.result(a.final_boards)
    assert bool(res.terminal.bool().all())
    assert torch.equal(res.diff, a.diff)
    hist = a.hist.cpu().numpy()
    assert hist[:129].sum() == n and hist[129:132].sum() == n
    assert hist[132] == int(a.plies.long().sum())
    np.testing.assert_array_equal(hist[:129], np.bincount(a.diff.cpu().numpy().astype(np.int64) + 64, minlength=129))
    # game length statistics of random play (mean 60.41, max 65)
    assert 60.0 < hist[132] / n < 61.0
    _oracle_full(a, n, 0x5EED, 0, 10)


@pytest.mark.parametrize("policy", ["greedy", "eval"])
def test_config5_full_size_vs_oracle(policy):
    """batch 1,048,576 with the 1-ply policies (config 5 and the eval player,
    default learner weights): every game bit-exact against the oracle, plus
    determinism, split invariance, terminal finals and histogram consistency.
    The oracle plays 1M greedy games in ~15-20 s and 1M eval games in
    ~30-40 s of 16 host threads on the GPU box (greedy ~3x, eval ~6x the
    random rate, measured on this image's host)."""
    from subproc_amd.params import DEFAULT_WEIGHTS
    w = DEFAULT_WEIGHTS if policy == "eval" else None
    pid = {"greedy": 1, "eval": 2}[policy]
    n = 1 << 20
    a = ops.rollout(n, 0x5EED, 0, policy, 10, device=DEV, weights=w)
    b = ops.rollout(n, 0x5EED, 0, policy, 10, device=DEV, weights=w)
    assert torch.equal(a.final_boards, b.final_boards) and torch.equal(a.hist, b.hist)
    k = 333_333
    h1 = ops.rollout(k, 0x5EED, 0, policy, 10, device=DEV, weights=w)
    h2 = ops.rollout(n - k, 0x5EED, k, policy, 10, device=DEV, weights=w)
    assert torch.equal(torch.cat([h1.final_boards, h2.final_boards]), a.final_boards)
    assert torch.equal(h1.hist + h2.hist, a.hist)
    res = ops.result(a.final_boards)
    assert bool(res.terminal.bool().all()) and torch.equal(res.diff, a.diff)
    hist = a.hist.cpu().numpy()
    assert hist[:129].sum() == n and hist[129:132].sum() == n
    assert hist[132] == int(a.plies.long().sum())
    np.testing.assert_array_equal(hist[:129], np.bincount(a.diff.cpu().numpy().astype(np.int64) + 64, minlength=129))
    _oracle_full(a, n, 0x5EED, pid, 10, weights=w)


def test_config4_global_histogram_equals_shards():
    """8,388,608 games in one launch == 8 rank-sized shards (the config-4 layout:
    rank r plays ids [r*2^20, (r+1)*2^20)), bit-exact: what the RCCL all-reduce
    of per-rank histograms must reproduce."""
    n = 1 << 20
    whole = ops.rollout(8 * n, 0x5EED, 0, device=DEV, want_boards=False, want_diff=False, want_plies=False)
    acc = torch.zeros_like(whole.hist)
    for r in range(8):
        ops.rollout(n, 0x5EED, r * n, hist=acc, device=DEV, want_boards=False, want_diff=False, want_plies=False)
    assert torch.equal(acc, whole.hist)
    assert int(whole.hist[:129].sum()) == 8 * n


def test_config4_histogram_vs_oracle():
    """The config-4 global histogram (8,388,608 random games, seed 0x5EED, ids
    0..8M-1: what the 8 ranks' RCCL all-reduce sums to) against the oracle
    playing the same 8M games on all host threads (~40 s of 16 threads on the
    GPU box).  Rule: game_runner.py:165-201 / board.py:192-209; the result rule
    of game_runner.py:194-199 fills bins 129-131."""
    n = 8 << 20
    whole = ops.rollout(n, 0x5EED, 0, device=DEV, want_boards=False, want_diff=False, want_plies=False)
    o = oracle.rollout(n, 0x5EED, 0, policy=0, n_random=10, n_threads=0)
    np.testing.assert_array_equal(whole.hist.cpu().numpy(), o["hist"])


def test_rollout_match_vs_oracle_and_equal_tables():
    from subproc_amd.params import DEFAULT_WEIGHTS
    n = 4096
    wr = np.random.default_rng(8).integers(-127, 128, (4, 9)).astype(np.int8)
    r = ops.rollout(n, 44, 1 << 22, "eval", 8, weights=DEFAULT_WEIGHTS, weights_white=wr, device=DEV)
    o = oracle.rollout(n, 44, 1 << 22, policy=2, n_random=8, weights=DEFAULT_WEIGHTS, weights_white=wr)
    assert (U(r.final_boards) == o["final_boards"]).all()
    assert (r.hist.cpu().numpy() == o["hist"]).all()
    # a match of a table against itself is the plain eval policy
    a = ops.rollout(n, 45, 0, "eval", 10, weights=wr, weights_white=wr, record_moves=True, device=DEV)
    b = ops.rollout(n, 45, 0, "eval", 10, weights=wr, record_moves=True, device=DEV)
    assert torch.equal(a.moves, b.moves) and torch.equal(a.hist, b.hist)


@pytest.mark.parametrize("n", [1, 63, 65, 1000])
def test_rollout_ragged_sizes_vs_oracle(n):
    for policy, pid in (("random", 0), ("greedy", 1)):
        r = ops.rollout(n, 31, 7, policy, 10, record_moves=True, device=DEV)
        o = oracle.rollout(n, 31, 7, policy=pid, n_random=10, record_moves=True)
        assert (r.moves.cpu().numpy() == o["moves"]).all(), (n, policy)
        assert (r.hist.cpu().numpy() == o["hist"]).all(), (n, policy)


def test_rollout_game_ids_wrap_2_64():
    """Game ids are u64 and wrap (game i uses id game_id0 + i mod 2^64)."""
    g0 = 2**64 - 10
    r = ops.rollout(32, 5, g0, device=DEV, record_moves=True)
    o = oracle.rollout(32, 5, g0, record_moves=True)
    assert (r.moves.cpu().numpy() == o["moves"]).all()
    tail = ops.rollout(22, 5, 0, device=DEV, record_moves=True)  # ids 0..21 == games 10..31 above
    assert torch.equal(tail.moves, r.moves[10:])


def test_concurrent_rollouts_on_two_streams():
    """Launches in flight together use separate work words (one per stream,
    ops.work_word): results equal the same launches run one after the other."""
    n = 1 << 18
    seq = [ops.rollout(n, 77, k * n, "random", device=DEV) for k in range(2)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for k, st in enumerate((s1, s2)):
        with torch.cuda.stream(st):
            outs.append(ops.rollout(n, 77, k * n, "random", device=DEV))
    torch.cuda.synchronize()
    for a, b in zip(seq, outs):
        assert torch.equal(a.final_boards, b.final_boards) and torch.equal(a.hist, b.hist)


def test_mixed_device_and_cpu_arguments_are_rejected():
    b, t, nt = ops.reset(8, "cuda")
    with pytest.raises(ValueError):
        ops.step(b, t.cpu(), torch.zeros(8, dtype=torch.uint8, device=DEV))
    with pytest.raises(ValueError):
        ops.rollout(8, 1, hist=torch.zeros(133, dtype=torch.int64), device=DEV)
    r = ops.rollout(8, 1, hist=torch.zeros(133, dtype=torch.int64, device=DEV), device="cuda")  # "cuda" == cuda:0
    assert int(r.hist[:129].sum()) == 8


def test_work_word_returns_to_zero_across_sizes():
    """A launch leaves its work word at 0 (the last dequeue resets it), so one
    word serves any sequence of launches on a stream: 130 launches of varying
    sizes and policies all equal their reference."""
    ref = {n: ops.rollout(n, 3, 1000, device=DEV, want_boards=False, want_plies=False).hist
           for n in (1, 64, 1000, 5000)}
    w = torch.zeros(1, dtype=torch.int64, device=DEV)
    for k in range(130):
        n = (1, 64, 1000, 5000)[k % 4]
        r = ops.rollout(n, 3, 1000, device=DEV, want_boards=False, want_plies=False, work=w)
        assert torch.equal(r.hist, ref[n]), (k, n)
        if k % 13 == 0:
            ops.rollout(777, 4, 0, "greedy", 10, device=DEV, work=w)
    assert int(w.item()) == 0


def test_many_rollouts_in_flight_on_several_streams():
    """96 launches (more than the 64 the r1 slot table allowed) in flight on 4
    streams, each stream with its own work word; stream 1 starts behind a
    sleep so later launches on the other streams overtake its earlier ones.
    Every launch equals the same launch run alone."""
    n = 3000
    ids = [(k * 7919) % 50000 for k in range(96)]
    ref = [ops.rollout(n, 21, g, device=DEV, want_diff=False, want_plies=False) for g in ids[:8]]
    streams = [torch.cuda.Stream() for _ in range(4)]
    torch.cuda.synchronize()
    with torch.cuda.stream(streams[1]):
        torch.cuda._sleep(50_000_000)  # ~20 ms: the other streams run ahead
    outs = []
    for k, g in enumerate(ids):
        with torch.cuda.stream(streams[k % 4]):
            outs.append(ops.rollout(n, 21, g, device=DEV, want_diff=False, want_plies=False))
    torch.cuda.synchronize()
    for k in range(8):
        assert torch.equal(outs[k].final_boards, ref[k].final_boards) and torch.equal(outs[k].hist, ref[k].hist), k
    for k in range(8, 96):
        assert int(outs[k].hist[:129].sum()) == n, k  # no game dropped
        if k % 8 == 0:
            alone = ops.rollout(n, 21, ids[k], device=DEV, want_diff=False, want_plies=False)
            assert torch.equal(outs[k].final_boards, alone.final_boards), k
    for st in streams:
        with torch.cuda.stream(st):
            assert int(ops.work_word(DEV).item()) == 0


def test_rollout_captured_in_a_graph_replays_correctly():
    """A captured oth_rollout needs no reset node: each replay finds its work
    word at 0 and leaves it at 0, so every replay plays all games; eager
    launches before and after the replays are unaffected."""
    n = 3000
    ref = ops.rollout(n, 9, 50, device=DEV)
    fb = torch.empty((n, 2), dtype=torch.int64, device=DEV)
    hist = torch.zeros(133, dtype=torch.int64, device=DEV)
    w = torch.zeros(1, dtype=torch.int64, device=DEV)
    from subproc_amd import _lib
    lib = _lib.load()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.oth_rollout(None, None, 9, 50, 0, 10, fb.data_ptr(), None, None, None, hist.data_ptr(),
                                   w.data_ptr(), n, st), "oth_rollout")
    for k in range(3):
        hist.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(fb, ref.final_boards), k
        assert torch.equal(hist, ref.hist), k
        assert int(w.item()) == 0
        mid = ops.rollout(n, 9, 50, device=DEV)
        assert torch.equal(mid.hist, ref.hist), k


def test_ops_rollout_graphs_replayed_concurrently():
    """ops.rollout under capture needs its own work word (a replay runs on the
    replaying stream, so two graphs that baked in one word would share a
    counter when replayed side by side); with one word per captured launch,
    two graphs replayed concurrently on two streams both play all their games."""
    n = 5000
    want = [ops.rollout(n, 11, k * n, device=DEV) for k in range(2)]
    words = [torch.zeros(1, dtype=torch.int64, device=DEV) for _ in range(2)]
    hists = [torch.zeros(133, dtype=torch.int64, device=DEV) for _ in range(2)]
    graphs, outs = [], []
    torch.cuda.synchronize()
    for k in range(2):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            with pytest.raises(RuntimeError, match="explicit work word"):
                ops.rollout(n, 11, k * n, device=DEV)
            outs.append(ops.rollout(n, 11, k * n, hist=hists[k], device=DEV, work=words[k]))
        graphs.append(g)
    streams = [torch.cuda.Stream(DEV) for _ in range(2)]
    for rep in range(4):
        for h in hists:
            h.zero_()
        torch.cuda.synchronize()
        for g, st in zip(graphs, streams):
            with torch.cuda.stream(st):
                g.replay()
        torch.cuda.synchronize()
        for k in range(2):
            assert torch.equal(outs[k].final_boards, want[k].final_boards), (rep, k)
            assert torch.equal(hists[k], want[k].hist), (rep, k)
            assert int(words[k].item()) == 0


def _high_mobility_boards(m, seed, iters=400):
    """Hill-climb random boards (single-square mutations kept when Black's
    mobility does not drop) to positions with 24..33 legal moves."""
    rng = np.random.default_rng(seed)
    occ = rng.integers(0, 2**64, m, dtype=np.uint64) & rng.integers(0, 2**64, m, dtype=np.uint64)
    nb = np.stack([occ & ~rng.integers(0, 2**64, m, dtype=np.uint64), np.zeros(m, np.uint64)], 1)
    nb[:, 1] = occ & ~nb[:, 0]
    black = np.full(m, 1, np.uint8)
    cur = np.bitwise_count(oracle.legal(nb, black)).astype(int)
    for _ in range(iters):
        bit = np.uint64(1) << rng.integers(0, 64, m).astype(np.uint64)
        kind = rng.integers(0, 3, m)
        nb2 = nb & ~bit[:, None]
        nb2[kind == 1, 0] |= bit[kind == 1]
        nb2[kind == 2, 1] |= bit[kind == 2]
        m2 = np.bitwise_count(oracle.legal(nb2, black)).astype(int)
        acc = m2 >= cur
        nb[acc], cur[acc] = nb2[acc], m2[acc]
    return nb, cur


@pytest.mark.parametrize("cap", [None, "0"])
def test_greedy_eval_coop_overflow_fallback_vs_oracle(cap, monkeypatch):
    """The cooperative choice (othello.hip coop_choose) cuts the wave's T
    children into 64 chunks of R = ceil(T / 64), found by a scan and a binary
    search, each walking parents' masks across parent boundaries; the per-lane
    choice (lane_choose) runs instead with OTH_COOP_CAP=0.  Start every game
    where the mover has >= 21 legal moves (chunks that start mid-parent and
    span several parents), both ways: all equal the oracle."""
    from subproc_amd.params import DEFAULT_WEIGHTS
    if cap is not None:
        monkeypatch.setenv("OTH_COOP_CAP", cap)
    nb, mob = _high_mobility_boards(4096, 12)
    assert mob.min() >= 21
    tt = np.full(len(nb), 1, np.uint8)
    for policy, pid, w in (("greedy", 1, None), ("eval", 2, DEFAULT_WEIGHTS)):
        r = ops.rollout(len(nb), 8, 0, policy, 0, start=B(nb[:, 0], nb[:, 1]), start_turn=T(tt), record_moves=True,
                        weights=w, device=DEV)
        o = oracle.rollout(len(nb), 8, 0, pid, 0, start=nb, start_turn=tt, record_moves=True, weights=w)
        assert (r.moves.cpu().numpy() == o["moves"]).all(), policy
        assert (r.hist.cpu().numpy() == o["hist"]).all(), policy
