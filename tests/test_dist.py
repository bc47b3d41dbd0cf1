"""N>1 path on CPU: world_size-2 gloo, disjoint game-id shards + one histogram
all_reduce.  The compute is injected (the C oracle, as checker) because this
container has no GPU; the sharding/reduction host logic is the product's."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from subproc_amd.dist import bench_game_id0, hist_summary, rollout_sharded, shard_range


def _oracle_fn(n, seed, game_id0, policy, n_random, hist):
    pid = {"random": 0, "greedy": 1}[policy]
    hist += torch.from_numpy(oracle.rollout(n, seed, game_id0, pid, n_random, n_threads=1)["hist"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, seed, out, bench_steps=0, steps=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if bench_steps:
        # bench.py's schedule: K steps of `total` games per rank, ids from
        # bench_game_id0, one histogram per step, summed and all-reduced once
        hist = torch.zeros(oracle.HIST_BINS, dtype=torch.int64)
        for s in range(bench_steps):
            _oracle_fn(total, seed, bench_game_id0(s, rank, world, total), "random", 10, hist)
        dist.all_reduce(hist, op=dist.ReduceOp.SUM)
        local = bench_steps * total
    else:
        hist, local = rollout_sharded(total, seed, rollout_fn=_oracle_fn, device="cpu", steps=steps)
    out[rank] = (hist.numpy().copy(), local)
    dist.destroy_process_group()


def _run(world, total, seed, bench_steps=0, steps=1):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), total, seed, out, bench_steps, steps), nprocs=world, join=True)
    return dict(out)


def test_bench_game_ids_tile_the_run():
    """bench.py step s on rank r plays [(s*world + r)*n, +n): over K steps and all
    ranks the ids are disjoint and cover [0, K*world*n) exactly."""
    n, K = 5, 4
    for world in (1, 2, 4, 8):
        ids = [g for s in range(K) for r in range(world)
               for g in range(bench_game_id0(s, r, world, n), bench_game_id0(s, r, world, n) + n)]
        assert sorted(ids) == list(range(K * world * n))


def test_world2_bench_schedule_equals_single_process():
    """The bench's N>1 reduction (per-step shards, one all-reduce at the end) ==
    one process over the same global ids, bit for bit."""
    n, K, seed = 37, 3, 0x5EED
    res = _run(2, n, seed, bench_steps=K)
    ref = oracle.rollout(2 * K * n, seed, 0)["hist"]
    for rank in (0, 1):
        np.testing.assert_array_equal(res[rank][0], ref)


def test_shard_range_partitions():
    for total in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(e - b for b, e in rs) - min(e - b for b, e in rs) <= 1


def test_world2_histogram_equals_single_process():
    total, seed = 301, 0x5EED
    res = _run(2, total, seed)
    ref = oracle.rollout(total, seed, 0)["hist"]
    for rank in (0, 1):
        np.testing.assert_array_equal(res[rank][0], ref)
    assert res[0][1] + res[1][1] == total
    s = hist_summary(ref)
    assert s["games"] == total and s["black_wins"] + s["white_wins"] + s["draws"] == total


def test_world2_pipelined_steps_equal_single_process():
    """rollout_sharded(steps=K): each rank's shard in K consecutive launches
    (ragged: 301 games over 2 ranks x 4 steps) == one process over the ids."""
    total, seed = 301, 0x5EED
    res = _run(2, total, seed, steps=4)
    ref = oracle.rollout(total, seed, 0)["hist"]
    for rank in (0, 1):
        np.testing.assert_array_equal(res[rank][0], ref)
    assert res[0][1] + res[1][1] == total


def test_batch_stats_payload_matches_per_book_rule():
    """learn_base.store_batch_stats quantities from the histogram == the same
    quantities computed per game from the terminal boards (correct win rule)."""
    from golden_io import load_npz
    from subproc_amd.dist import batch_stats_payload
    z = load_npz("rollout_random.npz")
    r = oracle.rollout(len(z["plies"]), int(z["seed"]), int(z["game_id0"]))
    nb = np.array([bin(int(b)).count("1") for b in z["final_black"]])
    nw = np.array([bin(int(w)).count("1") for w in z["final_white"]])
    d = nb - nw
    p = batch_stats_payload(r["hist"], "gpuA", "gpuB")
    assert p["gpuA_win_rate"] == (nb > nw).mean() and p["gpuB_win_rate"] == (nw > nb).mean()
    assert p["min_disc_diff"] == d.min() and p["max_disc_diff"] == d.max()
    assert abs(p["avg_disc_diff"] - d.mean()) < 1e-12
    assert p["diffs"] == sorted(d.tolist())
