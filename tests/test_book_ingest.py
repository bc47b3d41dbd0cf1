"""Book ingest, host side: books.pack_book_strings (Board.deserialize's view of
a board string, board.py:253-258), td.records_plan, and the CPU build of
oth_book_parse / oth_td_updates_records (oracle/othello_cpu_abi.c), pinned to
tests/golden/td_records.json -- the reference learner's own hash_from_book /
board_from_a_book over altered books (gen_golden.py td_records_fixtures).  CPU
only; the GPU twin is tests/test_gpu_ingest.py."""
import ctypes

import numpy as np
import pytest

import oracle
from golden_io import load_json
from subproc_amd import books, codec, td

P = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


def lib():
    return oracle.cpu_abi()


def test_pack_book_strings_rules():
    p = books.pack_book_strings(["OX", "O" * 64, ""])
    assert p.size == 192
    assert bytes(p[:64]).decode() == "OX" + books.OPENING_BOOK[2:]  # the rest keeps Board()'s squares
    assert bytes(p[64:128]).decode() == "O" * 64
    assert bytes(p[128:]).decode() == books.OPENING_BOOK
    with pytest.raises(IndexError):
        books.pack_book_strings(["-" * 65])  # row 8 does not exist
    q = books.pack_book_strings(["é" + "O" * 63, "中" + "X" * 63])
    assert q.size == 128 and q[0] == 0xE9 and q[64] == ord("?")  # one byte per character, never 'O'/'X'
    assert books.pack_book_strings([]).size == 0
    b, w = codec.deserialize_board(books.OPENING_BOOK)
    assert (b, w) == (0x0000000810000000, 0x0000001008000000)


def random_lines(n, seed):
    rnd = np.random.default_rng(seed)
    alphabet = np.frombuffer(b"OX-OX-OX-ox.*\x00\xff ", np.uint8)
    raw = alphabet[rnd.integers(0, len(alphabet), (n, 67))]
    raw[:, 64] = ord(" ")
    raw[:, 66] = ord("\n")
    return raw


@pytest.mark.parametrize("stride", [64, 66, 67, 80])
def test_cpu_parse_matches_codec(stride):
    n = 3000
    raw = random_lines(n, stride)
    text = np.zeros((n, stride), np.uint8)
    text[:, :min(stride, 67)] = raw[:, :stride]
    text = text.reshape(-1)
    b = np.zeros((n, 2), np.uint64)
    t = np.zeros(n, np.uint8)
    assert lib().oth_book_parse(P(text), stride, P(b), P(t) if stride >= 66 else None, n, None) == 0
    want = np.array([codec.deserialize_board(bytes(r[:64]).decode("latin-1")) for r in raw], np.uint64)
    np.testing.assert_array_equal(b, want)
    if stride >= 66:
        np.testing.assert_array_equal(t, [codec.turn_from_string(chr(c)) for c in raw[:, 65]])
    # argument checks
    assert lib().oth_book_parse(P(text), 63, P(b), None, n, None) != 0
    assert lib().oth_book_parse(P(text), 64, P(b), P(t), n, None) != 0  # the side needs stride >= 66
    assert lib().oth_book_parse(None, 64, P(b), None, 0, None) == 0


def cpu_state_map(bks, lam=td.LAMBDA, a=td.A):
    """update_from_records through the CPU build: parse, update stream, stable
    sort, per-key EMA."""
    strings, term, lam_idx, lam_pow = td.records_plan(bks, lam)
    n = len(strings)
    text = books.pack_book_strings(strings)
    rows = np.zeros((n, 2), np.uint64)
    assert lib().oth_book_parse(P(text), 64, P(rows), None, n, None) == 0
    keys, vals = np.zeros(2 * n, np.int64), np.zeros(2 * n)
    assert lib().oth_td_updates_records(P(rows), P(term), P(lam_idx), P(lam_pow), P(keys), P(vals), n, None) == 0
    order = np.argsort(keys, kind="stable")
    sk, sv = keys[order], vals[order]
    out = {}
    for k, v in zip(sk.tolist(), sv.tolist()):
        cur = out.get(k, 0.0)
        out[k] = v if cur == 0.0 else cur * (1 - a) + v * a
    return {td.hash_string(k): v for k, v in out.items()}


def test_cpu_records_pipeline_matches_reference_learner():
    fx = load_json("td_records.json")
    bks = [(i, b, {}) for i, b in enumerate(fx["books"])]
    assert set(fx["kinds"]) >= {"gaps", "repeats", "shuffled", "str_turns", "short", "chars", "random_boards"}
    assert cpu_state_map(bks) == dict(zip(fx["hash"], fx["value"]))


def test_records_plan_exponents_and_errors():
    bks = [(0, [{"book": "", "turn": "7"}, {"book": "", "turn": 9}, {"book": "", "turn": 7}], {}),
           (1, [{"book": "", "turn": 3}], {})]
    strings, term, lam_idx, lam_pow = td.records_plan(bks, 0.9)
    assert strings == ["", "", "", ""] and term.tolist() == [0, 0, 0, 3]
    # exponents 0, -2, 0, 0: l ** -2 as the learner's float power
    assert [lam_pow[i] for i in lam_idx] == [1.0, 0.9 ** -2, 1.0, 1.0]
    with pytest.raises(IndexError):
        td.records_plan([(0, [], {})])
    with pytest.raises(ValueError):
        td.records_plan([(0, [{"book": "", "turn": "x"}], {})])
