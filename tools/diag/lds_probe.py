"""A short program for PMC passes (diagnostic, GPU box): 1,048,576-game
rollouts of the random, greedy and eval policies (config 3 / config 5 / the
eval player), three launches each on one stream, outputs written as the bench
writes them (final boards, diff, plies).
    rocprofv3 --pmc <counters> -- python3 tools/diag/lds_probe.py [policy,...]"""
import os
import sys

sys.path.insert(0, os.getcwd())
if os.environ.get("PROBE_LIB"):  # an A/B build instead of the in-tree library
    from subproc_amd import _lib  # noqa: E402
    _lib.LIB_PATH = os.path.abspath(os.environ["PROBE_LIB"])
import torch  # noqa: E402

from subproc_amd import ops  # noqa: E402
from subproc_amd.params import DEFAULT_WEIGHTS  # noqa: E402

n = 1 << 20
for pol in (sys.argv[1].split(",") if len(sys.argv) > 1 else ("random", "greedy", "eval")):
    w = DEFAULT_WEIGHTS if pol == "eval" else None
    for k in range(3):
        ops.rollout(n, 0x5EED, (k + 1) * n, pol, 10, device="cuda", weights=w)
    torch.cuda.synchronize()
    print(pol, "done", flush=True)
