"""GameRunner matches in batches: the job an ElJemTask performs
(eljem_task.py:9-20 -> subproc.do_match, subproc.py:15-39 -> GameRunner,
game_runner.py:104-201), for n games at once on the GPU.

``do_matches(conf, params, n, seed)`` plays n games between player A -- the
eval policy with ``params`` (the table paramgen writes for the engine,
eljem_task.py:13-16) -- and player B, with the conf keys do_match reads:

  proc_n_rand_hands_for_a / _b   GameRunner's random-move budgets (each capped
                                 at N_RAND_HAND_UNTIL = 10, game_runner.py:115-119)
  proc_randomize_black_white     per game, A plays White with probability 1/2

and returns what the reference's recorder and learner see: the books of every
game (GameBooks: flat-file text and per-ply records), the meta GameRunner
stores with them (``{'proc_a': Black's name, 'proc_b': White's name,
'hamletparam': ...}``, game_runner.py:182-183), the winner tuple play_a_game
returns (194-199), and the batch statistics LearnBasePlus.store_batch_stats
derives from the books (learn_base.py:58-110).

The schedule runs inside the rollout kernel (oth_rollout_runner,
include/othello.h); its draws come from each game's counter RNG stream
(DESIGN.md §4), so a batch is reproducible from (seed, game ids) and any
split of the ids over launches or GPUs plays the same games.
"""
from collections import namedtuple

import numpy as np

from . import codec, ops, params, stats
from .books import GameBooks

MatchBatch = namedtuple("MatchBatch", "games books meta won stats a_black")

N_RAND_HAND_UNTIL = 10  # game_runner.py:6


def hamlet_param_line(name, policy, weights):
    """The 'verbose p' line of the GPU engine (subproc_amd.engine): what
    GameRunner.extract_hamlet_param stores as 'hamletparam' (game_runner.py:124-130)."""
    extra = " weights=%s" % params.as_weights(weights).reshape(-1).tolist() if policy == "eval" else ""
    return "%s policy=%s%s" % (name, policy, extra)


def do_matches(conf, weights_a=None, n=1, seed=0, game_id0=0, weights_b=None, policy="eval", name_a="Hamlet",
               name_b="GPU", device="cuda", record=True, win_rule="reference", store=None):
    """n GameRunner games between A (``weights_a``) and B (``weights_b``,
    default params.DEFAULT_WEIGHTS), both playing ``policy``.

    Game i is global id ``game_id0 + i`` (its book id).  ``record=True``
    replays every game into books (the recorder's view); the batch stats are
    computed from the terminal records as learn_books hands them to
    store_batch_stats (``win_rule`` as subproc_amd.stats), and written to
    ``store`` if given.  The reference's engine named 'Hamlet' provides
    'hamletparam'; here player A is that engine."""
    n_rand_a = int(conf.get("proc_n_rand_hands_for_a", 0))
    n_rand_b = int(conf.get("proc_n_rand_hands_for_b", 0))
    swap = int(conf.get("proc_randomize_black_white", 0)) == 1
    wa = params.DEFAULT_WEIGHTS if weights_a is None else weights_a
    wb = params.DEFAULT_WEIGHTS if weights_b is None else weights_b
    r = ops.rollout_runner(n, seed, game_id0, policy, wa, wb, n_rand_a, n_rand_b, swap, record_moves=record,
                           device=device)
    a_black = r.a_black.cpu().numpy().astype(bool)
    # extract_hamlet_param (game_runner.py:124-130): Black's engine first, then
    # White's, per game (the colours follow the swap draw)
    line = {"a": hamlet_param_line(name_a, policy, wa), "b": hamlet_param_line(name_b, policy, wb)}

    def hamlet(black, white):
        for who, name in (black, white):
            if name == "Hamlet":
                return line[who]
        return "No Hamlet"

    meta = []
    for ab in a_black:
        black, white = (("a", name_a), ("b", name_b)) if ab else (("b", name_b), ("a", name_a))
        meta.append({"proc_a": black[1], "proc_b": white[1], "hamletparam": hamlet(black, white)})
    diff = r.diff.cpu().numpy().astype(int)
    won = [("Black", m["proc_a"]) if d > 0 else (("White", m["proc_b"]) if d < 0 else ("None", ""))
           for d, m in zip(diff, meta)]
    books = GameBooks.from_rollout(r) if record else None
    # the terminal record of each book (book[0] after learn_books' reverse sort,
    # replearn.py:34-39) with its meta: store_batch_stats' input
    fin = ops.to_numpy_u64(r.final_boards).reshape(-1, 2)
    texts = codec.serialize_boards(fin)
    pl = r.plies.cpu().numpy().astype(int)
    side = ["-"] * n
    if books is not None:  # the side to move the recorder wrote with the terminal board
        last = books.pos.row_off + r.plies.long().clamp(max=ops.MOVES_STRIDE)
        side = ["O" if t == 1 else ("X" if t == 2 else "-") for t in books.pos.turn[last].cpu().tolist()]
    terminal = [(game_id0 + i, [{"book": t, "whosturn": side[i], "turn": int(pl[i]), "end": True}], meta[i])
                for i, t in enumerate(texts)]
    st = stats.store_batch_stats(terminal, store=store, win_rule=win_rule, device=device)
    return MatchBatch(r, books, meta, won, st, a_black)


def wins_of_a(batch):
    """Player A's wins / losses / draws over a MatchBatch (by colour and swap)."""
    d = batch.games.diff.cpu().numpy().astype(int)
    sign = np.where(batch.a_black, 1, -1) * np.sign(d)
    return int((sign > 0).sum()), int((sign < 0).sum()), int((sign == 0).sum())
