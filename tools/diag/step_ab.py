"""A/B of oth_step builds (config 2 steady state, 16M mid-game boards) — GPU box.

  python tools/diag/step_ab.py LIB_A.so LIB_B.so [reps]
Both libraries expose the product C-ABI.  Their outputs are compared bit for
bit on the same inputs, then the two are timed alternately (HIP events, 20
launches per sample) so clock drift hits both alike."""
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib, ops  # noqa: E402

paths = sys.argv[1:3]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
res, argt = _lib.SIGNATURES["oth_step"]
libs = []
for p in paths:
    L = ctypes.CDLL(os.path.abspath(p))
    L.oth_step.restype, L.oth_step.argtypes = res, argt
    libs.append(L)

n = 1 << 24
pos = ops.sample_midgame(n, 0x5EED, device="cuda")
s = torch.cuda.current_stream()


def outputs():
    return [torch.empty_like(pos.boards), torch.empty_like(pos.turn), torch.empty(n, dtype=torch.int64, device="cuda"),
            torch.empty(n, dtype=torch.int64, device="cuda"), torch.empty(n, dtype=torch.int8, device="cuda")]


outs = [outputs() for _ in libs]
args = [(pos.boards.data_ptr(), pos.turn.data_ptr(), pos.move.data_ptr(), o[0].data_ptr(), o[1].data_ptr(),
         o[2].data_ptr(), o[3].data_ptr(), o[4].data_ptr(), None, n, s.cuda_stream) for o in outs]
for L, a in zip(libs, args):
    assert L.oth_step(*a) == 0
torch.cuda.synchronize()
same = all(torch.equal(x, y) for x, y in zip(outs[0], outs[1]))
print("outputs identical:", same)
if not same:
    sys.exit(1)
# clock ramp: ~300 ms of launches before any sample
t_end = torch.cuda.Event(enable_timing=True)
w0 = torch.cuda.Event(enable_timing=True)
w0.record()
while True:
    for L, a in zip(libs, args):
        for _ in range(10):
            L.oth_step(*a)
    t_end.record()
    torch.cuda.synchronize()
    if w0.elapsed_time(t_end) > 300:
        break
for r in range(reps):
    for p, L, a in zip(paths, libs, args):
        for _ in range(3):
            L.oth_step(*a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            L.oth_step(*a)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print("%-28s bpc=%-3s %.1f us  %.2f TB/s" % (os.path.basename(p), os.environ.get("OTH_STEP_BLOCKS_PER_CU", "-"),
                                                  us, n * 52 / us / 1e6))
