"""Batch statistics: ``LearnBasePlus.store_batch_stats``
(learn_base.py:58-120) over books, and the same payload straight from a GPU
rollout.

The reference reads the terminal record of every book (``book[0]`` after
learn_books' reverse sort, replearn.py:34-39), deserializes it into a Board,
counts discs, and stores under the key ``['stats', <first book id>, <last
book id>]`` (learn_base.py:110)::

    {<proc_a>_win_rate, <proc_b>_win_rate, min_disc_diff, max_disc_diff,
     avg_disc_diff, params_used, diffs (sorted)}

Two entry points build that payload:

* :func:`store_batch_stats` takes the reference's own ``books`` list (book id,
  records, meta), decodes the terminal boards on the host and counts the discs
  of the whole batch in one ``oth_result`` launch.  Everything else follows
  learn_base.py line by line, including what a malformed book does: it is
  skipped from the point where it raised, but still counts in the rates'
  denominator ``len(books)``.
* :func:`rollout_batch_stats` takes the final boards a rollout left in HBM
  (``ops.rollout``): disc counts by ``oth_result``, the win rule, the sorted
  diffs and the extrema on the device, one copy to the host at the end.  Game
  ``i`` stands for book id ``game_id0 + i``.

Win rule.  learn_base.py:77 counts a White win when ``white_discs >
black_wins`` -- against the running count of Black wins, not Black's discs.
``win_rule="correct"`` (the default) uses ``white_discs > black_discs``, the
rule of the result histogram (game_runner.py:194-199); ``win_rule="reference"``
reproduces line 77 exactly, running count and all, for callers that compare
against payloads the reference stored.  The Slack report and the ranking
(learn_base.py:112-141) stay out of scope.
"""
import numpy as np
import torch

from . import codec, ops

WIN_RULES = ("correct", "reference")
_OPEN_BLACK = 0x0000000810000000  # Board() (board.py:22-27): deserialize writes over it
_OPEN_WHITE = 0x0000001008000000


def _check_rule(win_rule):
    if win_rule not in WIN_RULES:
        raise ValueError(f"win_rule must be one of {WIN_RULES}, got {win_rule!r}")


def stats_key(book_id_from, book_id_to):
    """The parameter-store key of a batch (learn_base.py:110)."""
    return ["stats", str(book_id_from), str(book_id_to)]


def _payload(black_name, white_name, black_wins, white_wins, n_books, diffs_sorted, params_used):
    """learn_base.py:90-109 from the batch's counts (diffs_sorted non-empty)."""
    return {
        black_name + "_win_rate": float(black_wins) / float(n_books),
        white_name + "_win_rate": float(white_wins) / float(n_books),
        "min_disc_diff": diffs_sorted[0],
        "max_disc_diff": diffs_sorted[-1],
        "avg_disc_diff": float(sum(diffs_sorted)) / float(n_books),
        "params_used": params_used,
        "diffs": diffs_sorted,
    }


PARAMS_ORDERS = ("sorted", "set")


def store_batch_stats(books, store=None, win_rule="correct", device="cuda", count_fn=None, params_order="sorted"):
    """LearnBasePlus.store_batch_stats(books) (learn_base.py:58-110).

    ``books``: [(book_id, records, meta), ...] as replearn.learn_books builds
    them; ``records[0]`` is the terminal record ``{'book', 'whosturn', 'turn',
    ...}``, ``meta`` holds 'proc_a', 'proc_b' and 'hamletparam'.  Writes the
    payload with ``store.hmset(key, payload)`` when a parameter store is given
    (parameter_store.py:38) and returns ``(key, payload)``.

    ``params_used`` joins the distinct 'hamletparam' values with ' / '.  The
    reference joins a ``set`` (learn_base.py:95), so its order is the set's
    iteration order, which CPython randomises per process for strings
    (PYTHONHASHSEED).  ``params_order="sorted"`` (the default) sorts them, a
    deterministic order; ``"set"`` joins a set built by the same ``add`` calls in
    the same order, which reproduces the reference's string exactly in the same
    interpreter and hash seed (tests/test_stats.py runs it under
    PYTHONHASHSEED=0 against tests/golden/batch_stats.json).
    ``count_fn(boards (n, 2) uint64) -> (n_black, n_white)`` replaces the
    device count (host tests only); by default the discs are counted by
    ``oth_result`` on ``device``.
    """
    _check_rule(win_rule)
    if params_order not in PARAMS_ORDERS:
        raise ValueError(f"params_order must be one of {PARAMS_ORDERS}, got {params_order!r}")
    # pass 1: the terminal boards (learn_base.py:69-71); a book that raises
    # here has no effect but its share of len(books)
    ok, boards = [], []
    for k, (book_id, book, meta) in enumerate(books):
        try:
            last = book[0]
            bl, wh = codec.deserialize_board(last["book"], _OPEN_BLACK, _OPEN_WHITE)
            last["whosturn"], last["turn"]  # noqa: B018  (deserialize reads both)
        except Exception as e:  # learn_base.py:85-88
            print("Exception occured while processing %d th book (%r)" % (book_id, e))
            continue
        ok.append(k)
        boards.append((bl, wh))
    if ok:
        b = np.array(boards, dtype=np.uint64).reshape(-1, 2)
        if count_fn is None:
            r = ops.result(ops.from_numpy_u64(b, device))
            nb, nw = r.n_black.cpu().tolist(), r.n_white.cpu().tolist()
        else:
            nb, nw = (list(map(int, v)) for v in count_fn(b))
    # pass 2, in book order (learn_base.py:72-84): a meta key that is missing
    # stops that book's bookkeeping where it raised, as the reference's try does
    black_wins = white_wins = 0
    disc_diff, book_ids, params = [], [], set()
    black_name, white_name = "black", "white"
    for j, k in enumerate(ok):
        book_id, _, meta = books[k]
        black_discs, white_discs = nb[j], nw[j]
        disc_diff.append(black_discs - white_discs)
        if black_discs > white_discs:
            black_wins += 1
        elif white_discs > (black_wins if win_rule == "reference" else black_discs):
            white_wins += 1
        book_ids.append(book_id)
        try:
            black_name = meta["proc_a"]
            white_name = meta["proc_b"]
            params.add(meta["hamletparam"])
        except Exception as e:  # learn_base.py:85-88
            print("Exception occured while processing %d th book (%r)" % (book_id, e))
    if not books:
        raise ZeroDivisionError("float division by zero")  # learn_base.py:90 on an empty batch
    if not disc_diff:
        raise ValueError("min() arg is an empty sequence")  # learn_base.py:92: no book was readable
    payload = _payload(black_name, white_name, black_wins, white_wins, len(books), sorted(disc_diff),
                       " / ".join(sorted(params) if params_order == "sorted" else params))
    key = stats_key(min(book_ids), max(book_ids))
    if store is not None:
        store.hmset(key, payload)
    return key, payload


def rollout_batch_stats(final_boards, game_id0=0, black_name="gpu_black", white_name="gpu_white", params_used="",
                        win_rule="correct", store=None):
    """The store_batch_stats payload of n games a rollout left in HBM
    (``final_boards`` (n, 2) int64 on the device, e.g. ``ops.rollout(...).final_boards``);
    game i is book id ``game_id0 + i``.  Returns ``(key, payload)`` and writes
    it to ``store`` if given.  ``params_used`` names the weight tables the
    games were played with (the reference's 'hamletparam' strings)."""
    _check_rule(win_rule)
    n = ops._n(final_boards)
    if n == 0:
        raise ZeroDivisionError("float division by zero")
    r = ops.result(final_boards)
    nb, nw = r.n_black.int(), r.n_white.int()
    bwin = nb > nw
    if win_rule == "correct":
        wwin = nw > nb
    else:  # learn_base.py:77: White's discs against the Black wins of the books before it
        bw = bwin.int()
        wwin = ~bwin & (nw > torch.cumsum(bw, 0) - bw)
    diffs = torch.sort(r.diff).values
    wins = torch.stack([bwin.sum(), wwin.sum()]).cpu().tolist()
    payload = _payload(black_name, white_name, wins[0], wins[1], n, diffs.cpu().tolist(), params_used)
    key = stats_key(game_id0, game_id0 + n - 1)
    if store is not None:
        store.hmset(key, payload)
    return key, payload


def rollout_books(final_boards, game_id0=0, black_name="gpu_black", white_name="gpu_white", params_used=""):
    """The ``books`` list learn_books would hand store_batch_stats for these games
    (terminal record only; host strings): for tests and for feeding GPU games
    through the reference-shaped path."""
    b = ops.to_numpy_u64(final_boards).reshape(-1, 2)
    texts = codec.serialize_boards(b)
    meta = {"proc_a": black_name, "proc_b": white_name, "hamletparam": params_used}
    return [(game_id0 + i, [{"book": t, "whosturn": "-", "turn": 0, "end": True}], dict(meta))
            for i, t in enumerate(texts)]
