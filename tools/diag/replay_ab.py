"""A/B of oth_replay builds (diagnostic, GPU box): per 262,144-game launch, the
kernel alone and with a zero fill of the position rows before it (what
ops.replay needs from a build that leaves rows past plies unwritten).
  python tools/diag/replay_ab.py LIB.so [LIB.so ...]"""
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib, ops  # noqa: E402

res, argt = _lib.SIGNATURES["oth_replay"]
libs = []
for p in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(p))
    L.oth_replay.restype, L.oth_replay.argtypes = res, argt
    libs.append((os.path.basename(p), L))
n = int(os.environ.get("REPLAY_N", 1 << 18))
r = ops.rollout(n, 7, 0, "random", record_moves=True, device="cuda")
b = torch.empty((n, 129, 2), dtype=torch.int64, device="cuda")
t = torch.empty((n, 129), dtype=torch.uint8, device="cuda")
e = torch.empty((n, 129), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
outs = {}
for name, L in libs:
    b.fill_(-1)
    assert L.oth_replay(None, None, r.moves.data_ptr(), r.plies.data_ptr(), b.data_ptr(), t.data_ptr(), e.data_ptr(), n,
                        st) == 0
    torch.cuda.synchronize()
    outs[name] = (b.clone(), t.clone(), e.clone())
for rep in range(3):
    for name, L in libs:
        for fill in (False, True):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                if fill:
                    b.zero_()
                L.oth_replay(None, None, r.moves.data_ptr(), r.plies.data_ptr(), b.data_ptr(), t.data_ptr(),
                             e.data_ptr(), n, st)
            e1.record()
            torch.cuda.synchronize()
            print("%-20s fill=%d  %.1f us" % (name, fill, e0.elapsed_time(e1) / 10 * 1e3))
names = list(outs)
pl = r.plies.long()
rows = torch.arange(129, device="cuda")[None, :] <= pl[:, None]
for nm in names[1:]:
    a0, a1 = outs[names[0]], outs[nm]
    same = torch.equal(a0[0][rows], a1[0][rows]) and torch.equal(a0[1], a1[1]) and torch.equal(a0[2], a1[2])
    print("rows <= plies, turn, end identical %s vs %s: %s" % (names[0], nm, same))
    print("  rows past plies zero in %s: %s" % (nm, bool((a1[0][~rows] == 0).all())))
