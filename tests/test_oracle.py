"""Pin the C oracle to the reference: every fixture produced by running the real
board.py (tests/golden/gen_golden.py) must be reproduced bit-for-bit.  CPU only."""
import numpy as np
import pytest

import oracle
from golden_io import ROLLOUT_FIXTURES, h, load_json, load_npz


def test_reset_matches_board_init():
    op = load_json("opening.json")
    b, t, nt = oracle.reset(3)
    assert (b[:, 0] == h(op["black"])).all() and (b[:, 1] == h(op["white"])).all()
    assert (t == op["turn"]).all() and (nt == op["nturn"]).all()


def test_opening_known_answers():
    op = load_json("opening.json")
    b = np.array([[h(op["black"]), h(op["white"])]], np.uint64)
    assert oracle.legal(b, [1])[0] == h(op["legal_black"])
    assert oracle.legal(b, [2])[0] == h(op["legal_white"])
    for m in op["moves"]:
        r = oracle.step(b, [op["turn"]], [m["sq"]], nturn=[0])
        assert r["ret"][0] == m["ret"]
        assert r["flips"][0] == h(m["flips"])
        assert r["boards"][0, 0] == h(m["black"]) and r["boards"][0, 1] == h(m["white"])
        assert r["turn"][0] == m["turn"] and r["nturn"][0] == m["nturn"]
    res = oracle.result(b)
    assert res["terminal"][0] == int(op["is_game_over"])


def test_midgame_every_code():
    z = load_npz("midgame_step.npz")
    n = len(z["black"])
    boards = np.stack([z["black"], z["white"]], 1)
    assert (oracle.legal(boards, z["turn"]) == z["legal"]).all()
    for code in range(65):
        r = oracle.step(boards, z["turn"], np.full(n, code, np.uint8), nturn=np.zeros(n, np.uint8))
        np.testing.assert_array_equal(r["ret"], z["ret"][:, code])
        np.testing.assert_array_equal(r["boards"][:, 0], z["next_black"][:, code])
        np.testing.assert_array_equal(r["boards"][:, 1], z["next_white"][:, code])
        np.testing.assert_array_equal(r["turn"], z["next_turn"][:, code])
        np.testing.assert_array_equal(r["nturn"], z["next_nturn"][:, code])
        np.testing.assert_array_equal(r["legal_next"], z["next_legal"][:, code])


def test_edges():
    for e in load_json("edges.json"):
        b = np.array([[h(e["black"]), h(e["white"])]], np.uint64)
        res = oracle.result(b)
        assert res["terminal"][0] == int(e["is_game_over"]), e["name"]
        assert res["n_black"][0] == e["n_black"] and res["n_white"][0] == e["n_white"]
        assert oracle.legal(b, [1])[0] == h(e["legal_black"]), e["name"]
        assert oracle.legal(b, [2])[0] == h(e["legal_white"]), e["name"]
        for s in e["steps"]:
            r = oracle.step(b, [e["turn"]], [s["code"]])
            assert r["ret"][0] == s["ret"], (e["name"], s["code"])
            assert r["boards"][0, 0] == h(s["black"]) and r["boards"][0, 1] == h(s["white"])
            assert r["turn"][0] == s["turn"]


def test_rng_known_answers():
    rng = load_json("rng.json")
    keys = [int(k, 16) for k in rng["game_keys"]]
    for g, k in zip((0, 1, 2, 1 << 20, (1 << 40) + 3), keys):
        assert oracle.game_key(rng["seed"], g) == k
    for i, v in enumerate(rng["draws_g0"]):
        assert oracle.rng_draw(keys[0], i + 1) == v


@pytest.mark.parametrize("name", ROLLOUT_FIXTURES)
def test_rollouts(name):
    z = load_npz(name + ".npz")
    n = len(z["plies"])
    from_mid = "from_mid" in name
    r = oracle.rollout(n, int(z["seed"]), int(z["game_id0"]), int(z["policy"]), int(z["n_random"]),
                       start=np.stack([z["start_black"], z["start_white"]], 1) if from_mid else None,
                       start_turn=z["start_turn"] if from_mid else None, record_moves=True,
                       weights=z.get("weights"), weights_white=z.get("weights_white"))
    np.testing.assert_array_equal(r["moves"], z["moves"])
    np.testing.assert_array_equal(r["plies"], z["plies"])
    np.testing.assert_array_equal(r["diff"], z["diff"])
    np.testing.assert_array_equal(r["final_boards"][:, 0], z["final_black"])
    np.testing.assert_array_equal(r["final_boards"][:, 1], z["final_white"])
    hist = r["hist"]
    assert hist[:129].sum() == n and hist[129:132].sum() == n and hist[132] == int(z["plies"].sum())
    np.testing.assert_array_equal(hist[:129], np.bincount(z["diff"].astype(np.int64) + 64, minlength=129))


def test_eval_values():
    """oracle_eval against the reference's counts() + the learner's linear model
    (eval_values.npz: default_value() weights and a random int8 table)."""
    z = load_npz("eval_values.npz")
    boards = np.stack([z["black"], z["white"]], 1)
    n = len(boards)
    for col, side in ((0, 1), (1, 2), (2, 0)):  # 'O', 'X', '-' (turn_from_string -> Empty)
        sides = np.full(n, side, np.uint8)
        np.testing.assert_array_equal(oracle.features(boards, sides), z["counts"][:, col])
        for wk, ek in (("weights_default", "eval_default"), ("weights_rand", "eval_rand")):
            np.testing.assert_array_equal(oracle.evaluate(boards, sides, z[wk]), z[ek][:, col])
    # every learner shard is exercised
    discs = np.array([bin(int(b) | int(w)).count("1") for b, w in boards])
    assert len({0 if d <= 16 else 1 if d <= 32 else 2 if d <= 48 else 3 for d in discs}) == 4


def test_sample_midgame():
    z = load_npz("sample_midgame.npz")
    n = len(z["move"])
    r = oracle.sample_midgame(n, int(z["seed"]))
    np.testing.assert_array_equal(r["boards"][:, 0], z["black"])
    np.testing.assert_array_equal(r["boards"][:, 1], z["white"])
    np.testing.assert_array_equal(r["turn"], z["turn"])
    np.testing.assert_array_equal(r["nturn"], z["nturn"])
    np.testing.assert_array_equal(r["move"], z["move"])


def test_rollout_split_invariance():
    """Global game ids make results independent of how the batch is split (the
    property multi-GPU sharding relies on)."""
    a = oracle.rollout(96, 7, 1000)
    b1 = oracle.rollout(40, 7, 1000)
    b2 = oracle.rollout(56, 7, 1040)
    np.testing.assert_array_equal(a["final_boards"], np.concatenate([b1["final_boards"], b2["final_boards"]]))
    np.testing.assert_array_equal(a["hist"], b1["hist"] + b2["hist"])


def test_books_and_features_vs_reference():
    """Book lines/records and counts() features from board.py + the reference
    learner module (tests/golden/books.json) reproduced by the oracle."""
    zs = {n: load_npz(n + ".npz") for n in ("rollout_random", "rollout_random_from_mid")}
    for bk in load_json("books.json"):
        z, g = zs[bk["source"]], bk["game"]
        rp = oracle.replay(z["moves"][g:g + 1], z["plies"][g:g + 1],
                           np.stack([z["start_black"], z["start_white"]], 1)[g:g + 1], z["start_turn"][g:g + 1])
        p = int(z["plies"][g])
        assert len(bk["lines"]) == p + 1
        for k in range(p + 1):
            bl, wh = rp["boards"][0, k]
            assert oracle.serialize_str(bl, wh, rp["turn"][0, k]) == bk["lines"][k]
            assert bool(rp["end"][0, k]) == bk["records"][k]["end"]
            for side, ref in ((1, bk["counts"][k][0]), (2, bk["counts"][k][1])):
                f = oracle.features(np.array([[bl, wh]], np.uint64), [side])[0]
                assert list(f) == ref, (bk["game"], k, side)


@pytest.mark.parametrize("name", ["rollout_runner_eval", "rollout_runner_greedy", "rollout_runner_eval_mid"])
def test_runner_schedule_fixtures(name):
    """GameRunner matches (colour draw, go_for's random-move coin per player)
    as gen_golden.py drives them through board.py: every move, final board,
    ply count and colour assignment."""
    z = load_npz(name + ".npz")
    n = len(z["plies"])
    o = oracle.rollout_runner(n, int(z["seed"]), int(z["game_id0"]), int(z["policy"]), z["weights_a"],
                              z["weights_b"], int(z["n_rand_a"]), int(z["n_rand_b"]), bool(z["swap"]),
                              start=np.stack([z["start_black"], z["start_white"]], 1), start_turn=z["start_turn"],
                              record_moves=True)
    np.testing.assert_array_equal(o["moves"], z["moves"])
    np.testing.assert_array_equal(o["final_boards"], np.stack([z["final_black"], z["final_white"]], 1))
    np.testing.assert_array_equal(o["plies"], z["plies"])
    np.testing.assert_array_equal(o["diff"], z["diff"])
    np.testing.assert_array_equal(o["a_black"], z["a_black"])
    if bool(z["swap"]):
        assert 0 < int(z["a_black"].sum()) < n  # both colour assignments occur
