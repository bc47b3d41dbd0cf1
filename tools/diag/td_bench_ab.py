"""bench.py's td_state_map line alone for one library (diagnostic, GPU box):
    python tools/diag/td_bench_ab.py LIB.so [reps]
prints the median / min / max ms of the third batch's update (bench._bench_td)."""
import argparse
import os
import sys

sys.path.insert(0, os.getcwd())
from subproc_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
import torch  # noqa: E402

import bench  # noqa: E402
from subproc_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
r = bench._bench_td(ops, torch, dev, argparse.Namespace(seed=0x5EED), reps=int(sys.argv[2]) if len(sys.argv) > 2 else 7)
print("%-14s fork=%s median %.3f ms (%.3f-%.3f)  %.3e updates/s" % (
    os.path.basename(sys.argv[1]), os.environ.get("OTH_TD_EMA_FORK", "0"), r["ms"], r["ms_min"], r["ms_max"],
    r["value"]), flush=True)
