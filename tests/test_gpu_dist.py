"""The N>1 host path with the HIP compute: two gloo ranks in their own
processes, both on cuda:0, each playing its shard of the global game ids
through subproc_amd.dist.rollout_sharded's default rollout (the HIP kernel),
then the histogram all-reduce.  Every rank's reduced histogram must equal one
process over the same global ids (results independent of GPU
count).  tests/test_dist.py covers the same host logic on CPU with the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, seed, policy, base, out, steps=1):
    import torch.distributed as dist

    from subproc_amd.dist import rollout_sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    hist, local = rollout_sharded(total, seed, policy, 10, device=torch.device("cuda", 0), game_id_base=base,
                                  steps=steps)
    out[rank] = (hist.cpu().numpy().copy(), local)
    dist.destroy_process_group()


@pytest.mark.parametrize("policy,steps", [("random", 1), ("greedy", 1), ("random", 7), ("eval", 3)])
def test_two_ranks_on_one_gpu_equal_one_process(policy, steps):
    """steps > 1: each rank's shard as pipelined launches on two streams
    (ops.rollout_batches) plus the ragged remainder."""
    from subproc_amd import ops

    total, seed, base = 200_003, 0x5EED, 1 << 33
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), total, seed, policy, base, out, steps), nprocs=2, join=True)
    ref = ops.rollout(total, seed, base, policy, 10, device="cuda:0").hist.cpu().numpy()
    assert sorted(v[1] for v in out.values()) == [total // 2, total - total // 2]
    for rank in (0, 1):
        np.testing.assert_array_equal(out[rank][0], ref)


@pytest.mark.parametrize("policy,streams,merge", [("random", 2, True), ("random", 2, False), ("random", 3, True),
                                                  ("greedy", 2, True), ("greedy", 3, False), ("eval", 1, True)])
def test_rollout_batches_equal_one_launch(policy, streams, merge, monkeypatch):
    """ops.rollout_batches: K pipelined batches == one launch over the same
    global ids, game for game (final boards, diff, plies) and histogram, with
    the batches merged into launches of up to ops.ROLLOUT_MERGE_GAMES games
    (here set so that 5 batches run as launches of 2, 2 and 1 batches) or one
    launch each."""
    from subproc_amd import ops

    n, K, seed, g0 = 40_009, 5, 0x5EED, (1 << 36) + 11
    monkeypatch.setattr(ops, "ROLLOUT_MERGE_GAMES", 2 * n + 5)
    a = ops.rollout_batches(n, K, seed, g0, policy, 10, device="cuda:0", streams=streams, want_boards=True,
                            want_diff=True, want_plies=True, merge=merge)
    b = ops.rollout(n * K, seed, g0, policy, 10, device="cuda:0")
    torch.cuda.synchronize()
    assert torch.equal(a.final_boards, b.final_boards)
    assert torch.equal(a.diff, b.diff) and torch.equal(a.plies, b.plies)
    assert torch.equal(a.hist, b.hist)
