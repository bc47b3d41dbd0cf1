"""Book ingest on the GPU: oth_book_parse (board strings / flat-file lines back
into bitboards, Board.deserialize of board.py:253-258) and the learner's state
map over books from any source (td.StateMap.update_from_records ->
oth_td_updates_records), against the CPU build of the same header, the board.py
books fixtures and the reference learner's fixtures (td_state.npz,
td_records.json)."""
import ctypes

import numpy as np
import pytest
import torch

import oracle
from golden_io import load_json, load_npz
from subproc_amd import books, ops, td
from subproc_amd.books import GameBooks

pytestmark = pytest.mark.gpu
DEV = "cuda"
P = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731


def random_lines(n, seed):
    rnd = np.random.default_rng(seed)
    alphabet = np.frombuffer(b"OX-OX-OX-ox.*\x00\xff ", np.uint8)
    raw = alphabet[rnd.integers(0, len(alphabet), (n, 67))]
    raw[:, 64] = ord(" ")
    raw[:, 66] = ord("\n")
    return raw


@pytest.mark.parametrize("stride,offset", [(64, 0), (64, 4), (64, 1), (67, 0), (67, 3), (80, 0), (96, 16),
                                           (100, 0), (128, 0), (130, 0), (66, 0)])
def test_parse_matches_cpu_build(stride, offset):
    """16-B aligned strings take the vector path, anything else byte loads;
    n is not a multiple of the block or of a wave"""
    n = 70001
    raw = random_lines(n, stride + offset)
    text = np.zeros((n, stride), np.uint8)
    text[:, :min(stride, 67)] = raw[:, :stride]
    flat = np.concatenate([np.zeros(offset, np.uint8), text.reshape(-1)])
    want_turn = stride >= 66
    dt = torch.from_numpy(flat).to(DEV)[offset:]
    b, t = ops.book_parse(dt, n, stride=stride, want_turn=want_turn)
    cb, ct = np.zeros((n, 2), np.uint64), np.zeros(n, np.uint8)
    host = np.ascontiguousarray(flat[offset:])
    assert oracle.cpu_abi().oth_book_parse(P(host), stride, P(cb), P(ct) if want_turn else None, n, None) == 0
    np.testing.assert_array_equal(ops.to_numpy_u64(b), cb)
    if want_turn:
        np.testing.assert_array_equal(t.cpu().numpy(), ct)
    e0, _ = ops.book_parse(dt[:0], 0)
    assert e0.shape == (0, 2)
    with pytest.raises(ValueError):
        ops.book_parse(dt, n + 1, stride=stride)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4097])
def test_parse_shortest_text(n):
    """a text that ends right after the last string's side character (no
    newline): no byte past it is read as a square or a side"""
    raw = random_lines(n, n)
    flat = raw.reshape(-1)[:(n - 1) * 67 + 66].copy()
    buf = torch.zeros(flat.size + 256, dtype=torch.uint8, device=DEV)
    buf[flat.size:] = ord("O")  # bytes past the text must not be read as squares or sides
    buf[:flat.size] = torch.from_numpy(flat).to(DEV)
    b, t = ops.book_parse(buf[:flat.size], n, stride=67, want_turn=True)
    cb, ct = np.zeros((n, 2), np.uint64), np.zeros(n, np.uint8)
    assert oracle.cpu_abi().oth_book_parse(P(flat), 67, P(cb), P(ct), n, None) == 0
    np.testing.assert_array_equal(ops.to_numpy_u64(b), cb)
    np.testing.assert_array_equal(t.cpu().numpy(), ct)


def test_parse_round_trips_gpu_books_and_flat_files(tmp_path):
    """the text the book emitter writes parses back to the replayed boards: the
    whole packed text in place (stride 67, with the side to move), the records'
    strings, and FlatFileRecorder files read back with books.read_flat_file"""
    r = ops.rollout(4096, 31, 0, "random", record_moves=True, device=DEV)
    gb = GameBooks.from_rollout(r)
    R = gb.pos.boards.shape[0]
    b, t = ops.book_parse(gb._text, R, stride=67, want_turn=True)
    assert torch.equal(b, gb.pos.boards) and torch.equal(t, gb.pos.turn)
    recs = [rec for g in range(0, 4096, 97) for rec in gb.records(g)]
    rows = torch.cat([gb.pos.boards[gb.game_rows(g)] for g in range(0, 4096, 97)])
    assert torch.equal(books.parse_book_strings([x["book"] for x in recs], DEV), rows)
    paths = gb.write_flat_files(str(tmp_path), games=[0, 5, 4095], black_name="Hamlet", white_name="GPU")
    for g, path in zip([0, 5, 4095], paths):
        bn, wn, fb, ft = books.read_flat_file(path, DEV)
        assert (bn, wn) == ("Hamlet", "GPU")
        assert torch.equal(fb, gb.pos.boards[gb.game_rows(g)]) and torch.equal(ft, gb.pos.turn[gb.game_rows(g)])


def test_parse_books_fixture():
    """the board.py records of books.json (FlatFileRecorder / RedisRecorder output)"""
    bj = load_json("books.json")
    strings = [rec["book"] for bk in bj for rec in bk["records"]]
    got = ops.to_numpy_u64(books.parse_book_strings(strings, DEV))
    host = books.pack_book_strings(strings)
    cb = np.zeros((len(strings), 2), np.uint64)
    assert oracle.cpu_abi().oth_book_parse(P(host), 64, P(cb), None, len(strings), None) == 0
    np.testing.assert_array_equal(got, cb)
    lines = "".join(line + "\n" for bk in bj for line in bk["lines"]).encode()
    b, t = ops.book_parse(torch.frombuffer(bytearray(lines), dtype=torch.uint8).to(DEV), len(strings), 67, True)
    np.testing.assert_array_equal(ops.to_numpy_u64(b), got)
    assert t.cpu().tolist() == [{"O": 1, "X": 2}.get(rec["whosturn"], 0) for bk in bj for rec in bk["records"]]


def test_state_map_from_records_matches_reference_learner():
    """td_records.json: altered books (gaps, repeats, shuffled records, string
    turns, short strings, other characters, random boards) through the
    reference's hash_from_book / board_from_a_book; in one batch and in three"""
    fx = load_json("td_records.json")
    want = dict(zip(fx["hash"], fx["value"]))
    bks = [(i, b, {}) for i, b in enumerate(fx["books"])]
    sm = td.StateMap(DEV)
    assert sm.update_from_records(bks) == 2 * sum(len(b) for b in fx["books"])
    assert sm.items() == want
    sm2 = td.StateMap(DEV)
    for lo, hi in ((0, 1), (1, 17), (17, len(bks))):
        sm2.update_from_records(bks[lo:hi])
    assert sm2.items() == want
    assert td.StateMap(DEV).update_from_records([]) == 0
    with pytest.raises(IndexError):
        td.StateMap(DEV).update_from_records([(0, [], {})])


def test_state_map_from_records_equals_from_books():
    """the 256 rollout_random games as learn_books hands their records over ==
    td_state.npz; and 2,048 GPU games: records path == replay path"""
    z = load_npz("rollout_random.npz")
    f = load_npz("td_state.npz")
    gb = GameBooks(torch.from_numpy(z["moves"]).to(DEV), torch.from_numpy(z["plies"]).to(DEV))
    bks = [(g, list(reversed(gb.records(g))), {}) for g in range(gb.n)]
    sm = td.StateMap(DEV)
    sm.update_from_records(bks)
    assert sm.items() == {h: float(v) for h, v in zip(f["hash"].tolist(), f["value"])}
    r = ops.rollout(2048, 41, 0, "random", record_moves=True, device=DEV)
    gb2 = GameBooks.from_rollout(r)
    a, b = td.StateMap(DEV), td.StateMap(DEV)
    a.update_from_books(gb2)
    b.update_from_records([(g, list(reversed(gb2.records(g))), {}) for g in range(gb2.n)])
    assert torch.equal(a.keys, b.keys) and torch.equal(a.values, b.values)
