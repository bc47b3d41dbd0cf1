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


def _worker(rank, world, port, total, seed, policy, base, out):
    import torch.distributed as dist

    from subproc_amd.dist import rollout_sharded

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    hist, local = rollout_sharded(total, seed, policy, 10, device=torch.device("cuda", 0), game_id_base=base)
    out[rank] = (hist.cpu().numpy().copy(), local)
    dist.destroy_process_group()


@pytest.mark.parametrize("policy", ["random", "greedy"])
def test_two_ranks_on_one_gpu_equal_one_process(policy):
    from subproc_amd import ops

    total, seed, base = 200_003, 0x5EED, 1 << 33
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), total, seed, policy, base, out), nprocs=2, join=True)
    ref = ops.rollout(total, seed, base, policy, 10, device="cuda:0").hist.cpu().numpy()
    assert sorted(v[1] for v in out.values()) == [total // 2, total - total // 2]
    for rank in (0, 1):
        np.testing.assert_array_equal(out[rank][0], ref)
