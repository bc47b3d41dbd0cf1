"""GPU-resident version of the reference's learning loop:
self-play with the current eval table -> books -> TD state map -> per-shard fit
-> new table, repeated.  Run on the GPU box:

    python tools/learn_loop.py [rounds] [games_per_round]

Reference counterpart: subproc.do_match games recorded as books
(game_recorder.py), replearn.learn_books -> ProgressPositionMovesLearn
(__update_state_for_a_book, fit_parameter, __store_parameters) -> paramgen.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from subproc_amd import dist, ops, params, td  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    games = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 18
    dev = torch.device("cuda", 0)
    w = params.DEFAULT_WEIGHTS.copy()
    sm = td.StateMap(dev)
    for r in range(rounds):
        t0 = time.perf_counter()
        ro = ops.rollout(games, 1000 + r, 0, "eval", 10, record_moves=True, weights=w, device=dev)
        pos = ops.replay(ro.moves, ro.plies)
        n_upd = sm.update(pos.boards, ro.plies)
        coef, icpt, n = sm.fit()
        w_new = params.from_coef(coef)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        s = dist.hist_summary(ro.hist)
        print("round %d: %d games (%.0f ms incl. fit), %d updates -> %d states; black win %.3f, avg diff %+.2f"
              % (r, games, dt * 1e3, n_upd, len(sm), s["black_win_rate"], s["avg_diff"]))
        print("  weights by shard:", [list(map(int, row)) for row in w_new])
        w = w_new
    # the learned table against the learner's default one, both colour assignments
    # (oth_rollout_match: the GPU counterpart of GameRunner's engine A vs engine B)
    for name, wb, ww in (("learned(B) vs default(W)", w, params.DEFAULT_WEIGHTS),
                         ("default(B) vs learned(W)", params.DEFAULT_WEIGHTS, w)):
        m = ops.rollout(games, 99, 1 << 40, "eval", 10, weights=wb, weights_white=ww, device=dev)
        s = dist.hist_summary(m.hist)
        print("match %s: black wins %.3f, white wins %.3f, draws %.3f" %
              (name, s["black_win_rate"], s["white_win_rate"], int(m.hist[131]) / s["games"]))


if __name__ == "__main__":
    main()
