"""A/B of two oth_rollout builds on the config-3 workload, without the bench's
histogram self-check (for diagnostic builds whose histogram is incomplete) --
GPU box.  python tools/diag/rollout_ab.py LIB_A.so LIB_B.so [reps]
Each sample: 20 launches of 1,048,576 random games on two streams, HIP events."""
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib  # noqa: E402

paths = sys.argv[1:3]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
res, argt = _lib.SIGNATURES["oth_rollout"]
libs = []
for p in paths:
    L = ctypes.CDLL(os.path.abspath(p))
    L.oth_rollout.restype, L.oth_rollout.argtypes = res, argt
    libs.append(L)
n = 1 << 20
main = torch.cuda.current_stream()
streams = [main, torch.cuda.Stream()]
bufs = [(torch.empty((n, 2), dtype=torch.int64, device="cuda"), torch.empty(n, dtype=torch.int8, device="cuda"),
         torch.empty(n, dtype=torch.uint8, device="cuda")) for _ in streams]
hist = torch.zeros(133, dtype=torch.int64, device="cuda")
works = torch.zeros(2, dtype=torch.int64, device="cuda")


def run(L, k0, count):
    e = torch.cuda.Event()
    e.record(main)
    streams[1].wait_event(e)
    for k in range(count):
        i = k % 2
        fb, df, pl = bufs[i]
        st = L.oth_rollout(None, None, 0x5EED, (k0 + k) * n, 0, 10, fb.data_ptr(), df.data_ptr(), pl.data_ptr(), None,
                           hist.data_ptr(), works[i:i + 1].data_ptr(), n, streams[i].cuda_stream)
        assert st == 0
    e2 = torch.cuda.Event()
    e2.record(streams[1])
    main.wait_event(e2)


for L in libs:
    run(L, 0, 10)
torch.cuda.synchronize()
for r in range(reps):
    for p, L in zip(paths, libs):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        run(L, 100 + r * 20, 20)
        e1.record(main)
        torch.cuda.synchronize()
        print("%-28s %.4f ms/step" % (os.path.basename(p), e0.elapsed_time(e1) / 20))
