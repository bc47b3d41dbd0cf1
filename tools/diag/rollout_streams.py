"""Diagnostic (NOT product code): do 1M-game rollout launches issued
round-robin on S streams (each step its own output buffers) fill the per-launch
tail that a single stream leaves idle?  Histograms must equal the 1-stream run.
    python tools/diag/rollout_streams.py [games] [steps]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from subproc_amd import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
lib = _lib.load()
dev = torch.device("cuda", 0)
streams = [torch.cuda.Stream(dev) for _ in range(4)]
bufs = [(torch.empty((n, 2), dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int8, device=dev),
         torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(4)]
works = torch.zeros(4, dtype=torch.int64, device=dev)  # one rollout work word per stream


def run(S, gid0):
    hists = torch.zeros((K, _lib.HIST_BINS), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(K):
        st = streams[s % S]
        fb, df, pl = bufs[s % S]
        _lib.check(lib.oth_rollout(None, None, 0x5EED, gid0 + s * n, 0, 10, fb.data_ptr(), df.data_ptr(),
                                   pl.data_ptr(), None, hists[s].data_ptr(), works[s % S:s % S + 1].data_ptr(), n,
                                   st.cuda_stream), "oth_rollout")
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return dt, hists.cpu()


for rep in range(3):
    ref = None
    for S in (1, 2, 3, 4):
        dt, h = run(S, rep * K * n)
        if ref is None:
            ref = h
        steps = int(h[:, 132].sum())
        print(f"rep {rep} streams {S}: {dt * 1e3 / K:.3f} ms/step  {steps / dt:.4e} env-steps/s  "
              f"hist {'identical' if torch.equal(h, ref) else 'DIFFERENT'}", flush=True)
