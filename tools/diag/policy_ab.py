"""A/B of rollout builds on one GPU box (diagnostic; run via gpurun).

  python tools/diag/policy_ab.py LIB_A.so LIB_B.so [...] [--policies greedy,eval] [--reps 5]

Every library exposes the product C-ABI.  For each policy, 1,048,576 games from
the opening per launch (config 5's workload), launches on one stream, timed
by HIP events; the libraries alternate launch by launch so clock drift hits
all alike.  Their histograms must be identical (same game ids)."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib  # noqa: E402
from subproc_amd.ops import _weights_ptr  # noqa: E402
from subproc_amd.params import DEFAULT_WEIGHTS  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("libs", nargs="+")
p.add_argument("--policies", default="greedy,eval")
p.add_argument("--reps", type=int, default=5)
p.add_argument("--games", type=int, default=1 << 20)
a = p.parse_args()

libs = []
for path in a.libs:
    L = ctypes.CDLL(os.path.abspath(path))
    for name in ("oth_rollout", "oth_rollout_eval"):
        res, argt = _lib.SIGNATURES[name]
        getattr(L, name).restype, getattr(L, name).argtypes = res, argt
    libs.append(L)
n = a.games
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
fb = torch.empty((n, 2), dtype=torch.int64, device=dev)
df = torch.empty(n, dtype=torch.int8, device=dev)
pl = torch.empty(n, dtype=torch.uint8, device=dev)
work = torch.zeros(1, dtype=torch.int64, device=dev)
wp = _weights_ptr(DEFAULT_WEIGHTS)


def launch(L, pol, gid, hist):
    if pol == "eval":
        rc = L.oth_rollout_eval(None, None, 0x5EED, gid, 10, wp, fb.data_ptr(), df.data_ptr(), pl.data_ptr(), None,
                                hist.data_ptr(), work.data_ptr(), n, st.cuda_stream)
    else:
        rc = L.oth_rollout(None, None, 0x5EED, gid, {"random": 0, "greedy": 1}[pol], 10, fb.data_ptr(), df.data_ptr(),
                           pl.data_ptr(), None, hist.data_ptr(), work.data_ptr(), n, st.cuda_stream)
    assert rc == 0, rc


for pol in a.policies.split(","):
    hists = [torch.zeros(133, dtype=torch.int64, device=dev) for _ in libs]
    for L, h in zip(libs, hists):
        launch(L, pol, 1 << 44, h)
    torch.cuda.synchronize()
    ok = all(torch.equal(hists[0], h) for h in hists[1:])
    print(pol, "histograms identical:", ok, flush=True)
    if not ok:
        sys.exit(1)
    times = [[] for _ in libs]
    for r in range(a.reps):
        for i, L in enumerate(libs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            h = torch.zeros(133, dtype=torch.int64, device=dev)
            e0.record(st)
            launch(L, pol, (1 << 44) + (r + 1) * n, h)
            e1.record(st)
            torch.cuda.synchronize()
            times[i].append((e0.elapsed_time(e1), int(h[132])))
    for path, L, t in zip(a.libs, libs, times):
        grid = "?"
        if hasattr(L, "oth_rollout_grid"):
            L.oth_rollout_grid.restype, L.oth_rollout_grid.argtypes = ctypes.c_int, [ctypes.c_int, ctypes.c_int64]
            grid = L.oth_rollout_grid({"random": 0, "greedy": 1, "eval": 2}[pol], n)
        ms = sorted(x[0] for x in t)
        med = ms[len(ms) // 2]
        steps = sum(x[1] for x in t) / len(t)
        print("%-8s %-28s median %.3f ms  min %.3f  %.3e env-steps/s  grid %s blocks" % (
            pol, os.path.basename(path), med, ms[0], steps / med * 1e3, grid), flush=True)
