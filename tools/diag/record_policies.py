"""Time ops.rollout with move records for each policy (262,144 games; GPU box).
Usage: python tools/diag/record_policies.py [tag]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import ops  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else ""
n = 1 << 18
for pol in ("random", "greedy", "eval"):
    for rec in (False, True):
        for _ in range(2):
            ops.rollout(n, 3, 0, pol, record_moves=rec)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = 5
        for k in range(reps):
            ops.rollout(n, 3, (k + 1) * n, pol, record_moves=rec)
        e1.record()
        torch.cuda.synchronize()
        print("%s %-6s record=%d  %.3f ms per launch" % (tag, pol, rec, e0.elapsed_time(e1) / reps), flush=True)
