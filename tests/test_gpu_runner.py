"""GameRunner matches on the GPU (oth_rollout_runner / ops.rollout_runner /
runner.do_matches): the colour draw of subproc.do_match and go_for's random-move
coin per player (game_runner.py:104-201, subproc.py:15-39), against the
fixtures gen_golden.py drove through board.py and against the C oracle."""
import numpy as np
import pytest
import torch

import oracle
from golden_io import RUNNER_FIXTURES, load_npz
from oracle import batch_stats as ref_stats

pytestmark = pytest.mark.gpu

from subproc_amd import ops, runner  # noqa: E402
from subproc_amd.params import DEFAULT_WEIGHTS  # noqa: E402

DEV = "cuda"
U = ops.to_numpy_u64


@pytest.mark.parametrize("name", RUNNER_FIXTURES)
def test_runner_fixtures(name):
    z = load_npz(name + ".npz")
    n = len(z["plies"])
    start = ops.from_numpy_u64(np.stack([z["start_black"], z["start_white"]], 1), DEV)
    r = ops.rollout_runner(n, int(z["seed"]), int(z["game_id0"]), ["random", "greedy", "eval"][int(z["policy"])],
                           z["weights_a"], z["weights_b"], int(z["n_rand_a"]), int(z["n_rand_b"]), bool(z["swap"]),
                           start=start, start_turn=torch.as_tensor(z["start_turn"]).to(DEV), record_moves=True,
                           device=DEV)
    np.testing.assert_array_equal(r.moves.cpu().numpy(), z["moves"])
    np.testing.assert_array_equal(U(r.final_boards), np.stack([z["final_black"], z["final_white"]], 1))
    np.testing.assert_array_equal(r.plies.cpu().numpy(), z["plies"])
    np.testing.assert_array_equal(r.diff.cpu().numpy(), z["diff"])
    np.testing.assert_array_equal(r.a_black.cpu().numpy(), z["a_black"])


@pytest.mark.parametrize("policy", ["greedy", "eval"])
@pytest.mark.parametrize("cap", [None, "0"])
def test_runner_vs_oracle_at_scale(policy, cap, monkeypatch):
    """8,192 matches (budgets 10 / 4, colours drawn) against the oracle, move
    for move; with OTH_COOP_CAP=0 (2,048 matches) every choice is made by its
    own lane (lane_choose) instead of the cooperative chunks."""
    if cap is not None:
        monkeypatch.setenv("OTH_COOP_CAP", cap)
    n = 8192 if cap is None else 2048
    wb = np.random.default_rng(3).integers(-127, 128, (4, 9)).astype(np.int8)
    r = ops.rollout_runner(n, 99, 1 << 36, policy, DEFAULT_WEIGHTS, wb, 10, 4, True, record_moves=True, device=DEV)
    o = oracle.rollout_runner(n, 99, 1 << 36, 1 if policy == "greedy" else 2, DEFAULT_WEIGHTS, wb, 10, 4, True,
                              record_moves=True)
    np.testing.assert_array_equal(r.moves.cpu().numpy(), o["moves"])
    np.testing.assert_array_equal(r.a_black.cpu().numpy(), o["a_black"])
    np.testing.assert_array_equal(r.hist.cpu().numpy(), o["hist"])
    assert 0.45 < o["a_black"].mean() < 0.55


def test_runner_split_invariance_and_budget_cap():
    """Two launches over halves of the ids play the games of one launch; a
    budget above 10 plays as 10 (N_RAND_HAND_UNTIL, game_runner.py:117-118)."""
    n = 8192
    one = ops.rollout_runner(n, 5, 1000, "eval", DEFAULT_WEIGHTS, DEFAULT_WEIGHTS, 10, 2, True, device=DEV)
    a = ops.rollout_runner(n // 2, 5, 1000, "eval", DEFAULT_WEIGHTS, DEFAULT_WEIGHTS, 10, 2, True, device=DEV)
    b = ops.rollout_runner(n // 2, 5, 1000 + n // 2, "eval", DEFAULT_WEIGHTS, DEFAULT_WEIGHTS, 10, 2, True,
                           device=DEV)
    assert torch.equal(torch.cat([a.final_boards, b.final_boards]), one.final_boards)
    assert torch.equal(torch.cat([a.a_black, b.a_black]), one.a_black)
    capped = ops.rollout_runner(n, 5, 1000, "eval", DEFAULT_WEIGHTS, DEFAULT_WEIGHTS, 37, 2, True, device=DEV)
    assert torch.equal(capped.final_boards, one.final_boards)
    # no swap: A is Black in every game
    ns = ops.rollout_runner(256, 5, 0, "greedy", None, None, 3, 3, False, device=DEV)
    assert bool((ns.a_black == 1).all())


def test_do_matches_books_meta_and_stats():
    """The ElJemTask-shaped batch: per-game meta names Black's and White's
    engine by the drawn colours, the winner tuples follow the discs, the books'
    terminal records are the final boards, and the batch stats equal
    learn_base.py's rule (restated in oracle/batch_stats.py) over those books."""
    conf = {"proc_n_rand_hands_for_a": 6, "proc_n_rand_hands_for_b": 2, "proc_randomize_black_white": 1}
    wa = np.random.default_rng(8).integers(-100, 100, (4, 9)).astype(np.int8)
    n = 512
    mb = runner.do_matches(conf, wa, n, seed=17, game_id0=300, name_b="GPU-default")
    o = oracle.rollout_runner(n, 17, 300, 2, wa, DEFAULT_WEIGHTS, 6, 2, True)
    np.testing.assert_array_equal(mb.a_black.astype(np.uint8), o["a_black"])
    np.testing.assert_array_equal(U(mb.games.final_boards), o["final_boards"])
    for g in range(n):
        ab = bool(o["a_black"][g])
        assert mb.meta[g]["proc_a"] == ("Hamlet" if ab else "GPU-default")
        assert mb.meta[g]["proc_b"] == ("GPU-default" if ab else "Hamlet")
        assert mb.meta[g]["hamletparam"].startswith("Hamlet policy=eval weights=")
        d = int(o["diff"][g])
        assert mb.won[g] == (("Black", mb.meta[g]["proc_a"]) if d > 0 else
                             (("White", mb.meta[g]["proc_b"]) if d < 0 else ("None", "")))
    for g in (0, 1, n - 1):
        recs = mb.books.records(g)
        assert recs[-1]["end"] and len(recs) == int(o["plies"][g]) + 1
    books = [(300 + g, [{"book": mb.books.records(g)[-1]["book"], "whosturn": mb.books.records(g)[-1]["whosturn"],
                         "turn": int(o["plies"][g]), "end": True}], mb.meta[g]) for g in range(n)]
    assert mb.stats == ref_stats.store_batch_stats(books, reference_rule=True)
    w, l, dr = runner.wins_of_a(mb)
    assert w + l + dr == n


def test_hamletparam_is_blacks_engine_first():
    """GameRunner.extract_hamlet_param (game_runner.py:124-130) asks Black's
    engine first: with both players named Hamlet the parameter line is the one
    of whoever played Black in that game (the colours follow the swap draw)."""
    conf = {"proc_randomize_black_white": 1}
    wa = np.full((4, 9), 3, np.int8)
    n = 64
    mb = runner.do_matches(conf, wa, n, seed=23, name_a="Hamlet", name_b="Hamlet")
    line_a = runner.hamlet_param_line("Hamlet", "eval", wa)
    line_b = runner.hamlet_param_line("Hamlet", "eval", DEFAULT_WEIGHTS)
    assert line_a != line_b
    assert 0 < int(mb.a_black.sum()) < n
    for g in range(n):
        assert mb.meta[g]["hamletparam"] == (line_a if mb.a_black[g] else line_b)
    mb = runner.do_matches(conf, wa, n, seed=23, name_a="GPU", name_b="Hamlet")
    assert all(m["hamletparam"] == line_b for m in mb.meta)
    mb = runner.do_matches(conf, wa, n, seed=23, name_a="X", name_b="Y")
    assert all(m["hamletparam"] == "No Hamlet" for m in mb.meta)
