"""§8f row 3 on the GPU: the store_batch_stats payload from HIP rollouts
(rollout_batch_stats: oth_result + device reductions) and from books
(store_batch_stats: one oth_result launch), against the restatement of
learn_base.py:58-109 (oracle/batch_stats.py) over the same games, and against
the games board.py itself played (rollout_* fixtures)."""
import numpy as np
import pytest
import torch

import oracle
from golden_io import load_npz
from oracle import batch_stats as ref

pytestmark = pytest.mark.gpu

from subproc_amd import ops, stats  # noqa: E402
from subproc_amd.params import DEFAULT_WEIGHTS  # noqa: E402

DEV = "cuda"


@pytest.mark.parametrize("rule", stats.WIN_RULES)
@pytest.mark.parametrize("name", ["rollout_random", "rollout_greedy"])
def test_fixture_games_from_the_kernel(name, rule):
    z = load_npz(name + ".npz")
    n = len(z["plies"])
    r = ops.rollout(n, int(z["seed"]), int(z["game_id0"]), ["random", "greedy"][int(z["policy"])], int(z["n_random"]),
                    device=DEV)
    fin = np.stack([z["final_black"], z["final_white"]], 1)
    np.testing.assert_array_equal(ops.to_numpy_u64(r.final_boards), fin)
    books = stats.rollout_books(ops.from_numpy_u64(fin, DEV), int(z["game_id0"]), "A", "B", "p")
    want = ref.store_batch_stats(books, rule == "reference")
    assert stats.rollout_batch_stats(r.final_boards, int(z["game_id0"]), "A", "B", "p", win_rule=rule) == want
    assert stats.store_batch_stats(books, win_rule=rule, device=DEV) == want


@pytest.mark.parametrize("policy", ["random", "greedy", "eval"])
def test_rollout_stats_vs_oracle_games(policy):
    n = 16384 if policy == "random" else 4096
    r = ops.rollout(n, 0x5EED, 1 << 20, policy, 10, device=DEV)
    pid = ["random", "greedy", "eval"].index(policy)
    o = oracle.rollout(n, 0x5EED, 1 << 20, pid, 10, weights=DEFAULT_WEIGHTS if pid == 2 else None)
    books = stats.rollout_books(ops.from_numpy_u64(o["final_boards"], DEV), 1 << 20, "gpu_black", "gpu_white", "t")
    for rule in stats.WIN_RULES:
        want = ref.store_batch_stats(books, rule == "reference")
        got = stats.rollout_batch_stats(r.final_boards, 1 << 20, params_used="t", win_rule=rule)
        assert got == want, rule
    # the histogram the kernel accumulated agrees with the payload (correct rule)
    h = r.hist.cpu().tolist()
    _, p = stats.rollout_batch_stats(r.final_boards, win_rule="correct")
    assert p["gpu_black_win_rate"] == h[129] / n and p["gpu_white_win_rate"] == h[130] / n
    assert p["diffs"] == [d - 64 for d in range(129) for _ in range(h[d])]


def test_full_size_config3_stats_and_store():
    n = 1 << 20
    r = ops.rollout(n, 0x5EED, 0, device=DEV)

    class Store(dict):
        def hmset(self, key, mapping):
            self[tuple(key)] = mapping

    s = Store()
    key, p = stats.rollout_batch_stats(r.final_boards, 0, win_rule="reference", store=s)
    assert key == ["stats", "0", str(n - 1)] and s[tuple(key)] is p
    assert len(p["diffs"]) == n and p["diffs"] == sorted(p["diffs"])
    h = r.hist.cpu().tolist()
    assert p["gpu_black_win_rate"] == h[129] / n
    assert p["min_disc_diff"] == min(d - 64 for d in range(129) if h[d])
    _, pc = stats.rollout_batch_stats(r.final_boards, 0, win_rule="correct")
    assert pc["gpu_white_win_rate"] == h[130] / n
    # line 77's running count over all 1M games, restated in numpy: once 64
    # Black wins are in, no White disc count can exceed it
    fin = ops.to_numpy_u64(r.final_boards)
    nb = np.unpackbits(fin[:, 0:1].view(np.uint8), axis=1).sum(1)
    nw = np.unpackbits(fin[:, 1:2].view(np.uint8), axis=1).sum(1)
    bw = nb > nw
    before = np.cumsum(bw) - bw
    assert p["gpu_white_win_rate"] == int((~bw & (nw > before)).sum()) / n
    # a strided sample of the same games through the restated learner
    idx = np.arange(0, n, 1021)
    fin = ops.to_numpy_u64(r.final_boards)[idx]
    books = stats.rollout_books(ops.from_numpy_u64(fin, DEV))
    sub = torch.as_tensor(idx).to(DEV)
    for rule in stats.WIN_RULES:
        assert stats.rollout_batch_stats(r.final_boards[sub], win_rule=rule) == ref.store_batch_stats(
            books, rule == "reference")


def test_store_batch_stats_vs_reference_payload_device_count():
    """tests/golden/batch_stats.json (learn_base.py:58-110 run from the
    reference): the books' discs counted by oth_result on the GPU, every field
    of the key and payload equal (params_used up to the set order, which
    tests/test_stats.py pins byte for byte under the generator's hash seed)."""
    from golden_io import load_json

    for case in load_json("batch_stats.json")["cases"]:
        books = [(i, r, m) for i, r, m in case["books"]]
        key, payload = stats.store_batch_stats(books, win_rule="reference", device=DEV)
        want = dict(case["payload"])
        want["params_used"] = " / ".join(sorted(want["params_used"].split(" / ")))
        assert key == case["key"], case["name"]
        assert payload == want, case["name"]
