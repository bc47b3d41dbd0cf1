"""§8f row 3 on the host: subproc_amd.stats.store_batch_stats against the
line-for-line restatement of learn_base.py:58-109 (oracle/batch_stats.py),
disc counts injected (the device count is tests/test_gpu_stats.py's)."""
import numpy as np
import pytest

from golden_io import load_npz
from oracle import batch_stats as ref
from subproc_amd import codec, stats


def _popcount(a):
    a = np.ascontiguousarray(a, np.uint64)
    return np.unpackbits(a.view(np.uint8).reshape(-1, 8), axis=1).sum(axis=1)


def count(b):
    return _popcount(b[:, 0]), _popcount(b[:, 1])


def _books_from_finals(black, white, id0=0, meta=None):
    texts = codec.serialize_boards(np.stack([black, white], 1))
    meta = meta or {"proc_a": "A", "proc_b": "B", "hamletparam": "p0"}
    return [(id0 + i, [{"book": t, "whosturn": "O", "turn": 60, "end": True}], dict(meta)) for i, t in enumerate(texts)]


@pytest.mark.parametrize("rule", stats.WIN_RULES)
@pytest.mark.parametrize("name", ["rollout_random", "rollout_greedy", "rollout_random_from_mid"])
def test_fixture_games_vs_restated_learn_base(name, rule):
    z = load_npz(name + ".npz")
    books = _books_from_finals(z["final_black"], z["final_white"], int(z["game_id0"]))
    want = ref.store_batch_stats(books, reference_rule=rule == "reference")
    got = stats.store_batch_stats(books, win_rule=rule, count_fn=count)
    assert got == want
    assert got[1]["diffs"] == sorted(z["diff"].astype(int).tolist())  # board.py's own diffs


def test_reference_rule_differs_where_line_77_bites():
    # a Black win (63-1), then two draws (32-32, 8-8): line 77 compares White's
    # discs with the one Black win so far and counts both draws as White wins
    full = (1 << 64) - 1
    half = (1 << 32) - 1
    black = np.array([full ^ 1, half, 0x00000000000000FF], np.uint64)
    white = np.array([1, full ^ half, 0x000000000000FF00], np.uint64)
    books = _books_from_finals(black, white)
    k1, p_ref = stats.store_batch_stats(books, win_rule="reference", count_fn=count)
    k2, p_ok = stats.store_batch_stats(books, win_rule="correct", count_fn=count)
    assert p_ref == ref.store_batch_stats(books, True)[1]
    assert p_ok == ref.store_batch_stats(books, False)[1]
    assert p_ref["B_win_rate"] == pytest.approx(2 / 3) and p_ok["B_win_rate"] == 0.0
    assert k1 == k2 == ["stats", "0", "2"]


def test_malformed_books_follow_the_reference_try():
    rng = np.random.default_rng(0)
    bl = rng.integers(0, 2**64, 12, dtype=np.uint64)
    wh = rng.integers(0, 2**64, 12, dtype=np.uint64) & ~bl
    books = _books_from_finals(bl, wh, id0=100)
    books[1] = (101, [], books[1][2])                                         # empty book: skipped
    books[2][1][0]["book"] = books[2][1][0]["book"] + "O"                      # 65 cells: IndexError
    books[3][1][0]["book"] = "XXXXOOOO"                                        # short: over Board()
    del books[4][1][0]["whosturn"]                                             # KeyError before counting
    books[5] = (105, books[5][1], {"proc_a": "C"})                            # counted; names stop at proc_b
    books[6] = (106, books[6][1], None)                                       # counted; meta unreadable
    books[7] = (107, books[7][1], {"proc_a": "D", "proc_b": "E", "hamletparam": "p1"})
    books[8][1][0]["book"] = "".join(rng.choice(list("OX-?o "), 64))          # other chars -> Empty
    for rule in stats.WIN_RULES:
        got = stats.store_batch_stats(books, win_rule=rule, count_fn=count)
        assert got == ref.store_batch_stats(books, rule == "reference")
    assert got[1]["params_used"] == "p0 / p1"


def test_store_is_written_and_errors_match():
    class Store:
        def __init__(self):
            self.d = {}

        def hmset(self, key, mapping):
            self.d[tuple(key)] = mapping

    books = _books_from_finals(np.array([0xFF], np.uint64), np.array([0xFF00], np.uint64), id0=7)
    s = Store()
    key, payload = stats.store_batch_stats(books, store=s, count_fn=count)
    assert s.d == {("stats", "7", "7"): payload}
    with pytest.raises(ZeroDivisionError):
        stats.store_batch_stats([], count_fn=count)
    with pytest.raises(ValueError):
        stats.store_batch_stats([(1, [], {})], count_fn=count)
    with pytest.raises(ValueError):
        stats.store_batch_stats(books, win_rule="other", count_fn=count)


# ---------------------------------------------------------------------------
# pinned to the reference itself: tests/golden/batch_stats.json holds the
# (key, payload) learn_base.py:58-110 handed its parameter store's hmset for
# each batch of books, run from /root/reference by gen_golden.py
# ---------------------------------------------------------------------------
def _ref_cases():
    from golden_io import load_json
    return load_json("batch_stats.json")


def _books(case):
    return [(i, recs, meta) for i, recs, meta in case["books"]]


def _sorted_params(payload):
    p = dict(payload)
    p["params_used"] = " / ".join(sorted(p["params_used"].split(" / ")))
    return p


@pytest.mark.parametrize("name", [c["name"] for c in _ref_cases()["cases"]])
def test_store_batch_stats_vs_reference_payload(name):
    """Every field of the reference's payload and its key, with win_rule
    'reference'; params_used up to the set order (sorted on our side)."""
    case = next(c for c in _ref_cases()["cases"] if c["name"] == name)
    key, payload = stats.store_batch_stats(_books(case), win_rule="reference", count_fn=count)
    assert key == case["key"]
    assert payload == _sorted_params(case["payload"])
    # the restatement the other tests check against agrees with the reference too
    assert ref.store_batch_stats(_books(case), reference_rule=True) == (case["key"], _sorted_params(case["payload"]))


def test_store_batch_stats_byte_exact_in_the_reference_hash_order():
    """params_order='set' joins the set as learn_base.py:95 does: in an
    interpreter with the generator's PYTHONHASHSEED every (key, payload) equals
    the reference's byte for byte (as JSON), params_used order included."""
    import json
    import os
    import subprocess
    import sys
    d = _ref_cases()
    here = os.path.dirname(os.path.abspath(__file__))
    code = r'''
import json, sys
sys.path[:0] = [%r, %r]
import numpy as np
from golden_io import load_json
from subproc_amd import stats
def count(b):
    a = np.ascontiguousarray(b, np.uint64)
    pc = lambda v: np.unpackbits(v.view(np.uint8).reshape(-1, 8), axis=1).sum(axis=1)
    return pc(a[:, 0].copy()), pc(a[:, 1].copy())
out = []
for c in load_json("batch_stats.json")["cases"]:
    books = [(i, r, m) for i, r, m in c["books"]]
    key, payload = stats.store_batch_stats(books, win_rule="reference", count_fn=count, params_order="set")
    out.append(json.dumps([key, payload]) == json.dumps([c["key"], c["payload"]]))
print(json.dumps(out))
''' % (here, os.path.dirname(here))
    env = dict(os.environ, PYTHONHASHSEED=d["pythonhashseed"])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1]) == [True] * len(d["cases"])
