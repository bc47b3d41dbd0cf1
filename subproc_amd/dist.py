"""Multi-GPU self-play: one process per GPU, disjoint global game-id ranges,
ONE all_reduce(SUM) of the int64[133] win/score histogram (RCCL over xGMI with
backend "nccl"; gloo for CPU tests).

Replaces the reference's job fan-out (Resque/pyres queues on Redis,
replearn.py:78-86 -> eljem_worker.py:10 -> subproc.do_match) for the env path:
games are independent, so there is no data-path collective; the only exchange
is the episode-count/score reduction.
"""
import torch
import torch.distributed as dist

from ._lib import HIST_BINS


def shard_range(total, rank, world):
    """Contiguous [begin, end) of `total` games for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def bench_game_id0(step, rank, world, n):
    """First global game id of bench step `step` on `rank` (bench.py): step s
    plays ids [(s*world + r)*n, +n) on rank r, so every (step, rank) pair gets
    fresh, disjoint games and the ids of steps 0..K-1 over all ranks tile
    [0, K*world*n) exactly (tests/test_dist.py)."""
    return (step * world + rank) * n


def rollout_sharded(total_games, seed, policy="random", n_random=10, group=None, rollout_fn=None, device=None,
                    game_id_base=0, steps=1, streams=2):
    """Play `total_games` games split over the ranks of `group`; returns
    (global histogram int64[133] on every rank, local game count).

    Game g (global id game_id_base + g) always uses the same RNG stream, so the
    reduced histogram is identical for any world size (bit-exact check of the
    all-reduce path: tests/test_dist.py).  `rollout_fn(n, seed, game_id0,
    policy, n_random, hist)` defaults to the HIP kernel (subproc_amd.ops.rollout).

    steps > 1 splits the rank's range into `steps` consecutive launches
    pipelined over `streams` HIP streams (ops.rollout_batches: the repeated
    launches of bench.py's timed loop); the histogram is the same.  With a
    custom `rollout_fn` the chunks are played one call each, in order.
    """
    if steps < 1:
        raise ValueError("steps must be >= 1")
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    begin, end = shard_range(total_games, rank, world)
    if rollout_fn is None and device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    hist = torch.zeros(HIST_BINS, dtype=torch.int64, device=device)
    local = end - begin
    if local > 0:
        if rollout_fn is None:
            from . import ops
            per, rest = divmod(local, steps)
            if steps == 1 or streams == 1:
                # one launch per chunk on the caller's stream (no side stream,
                # no fork/join events: capturable, as before round 4)
                for c in range(steps):
                    b, e = shard_range(local, c, steps)
                    if e > b:
                        ops.rollout(e - b, seed, game_id_base + begin + b, policy, n_random, hist=hist,
                                    device=device, want_boards=False, want_diff=False, want_plies=False)
            else:
                if per:  # `steps` equal launches, then the remainder
                    ops.rollout_batches(per, steps, seed, game_id_base + begin, policy, n_random, hist=hist,
                                        device=device, streams=streams)
                if rest:
                    ops.rollout(rest, seed, game_id_base + begin + per * steps, policy, n_random, hist=hist,
                                device=device, want_boards=False, want_diff=False, want_plies=False)
        else:
            for c in range(steps):
                b, e = shard_range(local, c, steps)
                if e > b:
                    rollout_fn(e - b, seed, game_id_base + begin + b, policy, n_random, hist)
    if world > 1:
        reduce_histogram(hist, group)
    return hist, local


def reduce_histogram(hist, group=None):
    """The one collective: all_reduce(SUM) of the int64[133] histogram, in
    place.  RCCL ("nccl") reduces the device tensor where it lies; a gloo
    group (CPU tests, or ranks sharing one GPU) reduces a host copy."""
    if hist.is_cuda and dist.get_backend(group) == "gloo":
        h = hist.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        hist.copy_(h)
    else:
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    return hist


def hist_summary(hist):
    """Batch statistics from the histogram (learn_base.py:58-109 quantities,
    with the correct white-win rule, not learn_base.py:77's comparison bug)."""
    h = hist.tolist() if isinstance(hist, torch.Tensor) else list(hist)
    games = sum(h[:129])
    diffs = [d - 64 for d in range(129) if h[d]]
    return dict(games=games, black_wins=h[129], white_wins=h[130], draws=h[131], plies=h[132],
                black_win_rate=h[129] / games if games else 0.0, white_win_rate=h[130] / games if games else 0.0,
                avg_diff=sum((d - 64) * h[d] for d in range(129)) / games if games else 0.0,
                min_diff=min(diffs) if diffs else 0, max_diff=max(diffs) if diffs else 0)


def batch_stats_payload(hist, black_name="black", white_name="white", params_used=""):
    """The payload LearnBase.store_batch_stats stores (learn_base.py:91-109),
    computed from the GPU histogram instead of per-book Board.deserialize:
    '<black>_win_rate', '<white>_win_rate', min/max/avg disc diff, and the
    sorted per-game disc diffs (expanded from the histogram counts).
    Wins use the correct rule: white wins iff white_discs > black_discs
    (learn_base.py:77 compares against the running black-win count)."""
    h = hist.tolist() if isinstance(hist, torch.Tensor) else list(hist)
    s = hist_summary(h)
    if s["games"] == 0:
        raise ValueError("empty batch (learn_base.py divides by len(books))")
    diffs = [d - 64 for d in range(129) for _ in range(h[d])]
    return {black_name + "_win_rate": s["black_win_rate"], white_name + "_win_rate": s["white_win_rate"],
            "min_disc_diff": s["min_diff"], "max_disc_diff": s["max_diff"], "avg_disc_diff": s["avg_diff"],
            "params_used": params_used, "diffs": diffs}
