"""Config 2's launch floor on the GPU box: back-to-back launches of oth_step over
65,536 boards against launches of oth_reset (stores only, no loads, no VALU
to speak of) and oth_legal over the same boards, plain and captured in a HIP
graph.  The gap between step and reset is what the step kernel itself costs
at this size.

  python tools/diag/launch_floor.py [LIB.so ...]
Extra libraries (diagnostic builds with the same C-ABI) add their step lines."""
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib, ops  # noqa: E402

lib = _lib.load()
n = int(os.environ.get("LF_N", 65536))
pos = ops.sample_midgame(n, 0x5EED, device="cuda")
bo, to = torch.empty_like(pos.boards), torch.empty_like(pos.turn)
fl, ln = torch.empty(n, dtype=torch.int64, device="cuda"), torch.empty(n, dtype=torch.int64, device="cuda")
rt = torch.empty(n, dtype=torch.int8, device="cuda")
nt = torch.empty(n, dtype=torch.uint8, device="cuda")


extra = []
for path in sys.argv[1:]:
    L = ctypes.CDLL(os.path.abspath(path))
    L.oth_step.restype, L.oth_step.argtypes = _lib.SIGNATURES["oth_step"]
    extra.append((os.path.basename(path), L))


def calls(st):
    d = {
        "reset": lambda: lib.oth_reset(bo.data_ptr(), to.data_ptr(), nt.data_ptr(), n, st),
        "legal": lambda: lib.oth_legal(pos.boards.data_ptr(), pos.turn.data_ptr(), ln.data_ptr(), n, st),
        "step": lambda: lib.oth_step(pos.boards.data_ptr(), pos.turn.data_ptr(), pos.move.data_ptr(), bo.data_ptr(),
                                     to.data_ptr(), fl.data_ptr(), ln.data_ptr(), rt.data_ptr(), None, n, st),
        "step-nolegal": lambda: lib.oth_step(pos.boards.data_ptr(), pos.turn.data_ptr(), pos.move.data_ptr(),
                                             bo.data_ptr(), to.data_ptr(), fl.data_ptr(), None, rt.data_ptr(), None,
                                             n, st),
    }
    for name, L in extra:
        d["step:" + name] = (lambda L=L: L.oth_step(pos.boards.data_ptr(), pos.turn.data_ptr(), pos.move.data_ptr(),
                                                    bo.data_ptr(), to.data_ptr(), fl.data_ptr(), ln.data_ptr(),
                                                    rt.data_ptr(), None, n, st))
    return d


K = 400
s = torch.cuda.current_stream()
for name, fn in calls(s.cuda_stream).items():
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        fn()
    e1.record()
    torch.cuda.synchronize()
    plain = e0.elapsed_time(e1) / K * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fns = calls(torch.cuda.current_stream().cuda_stream)
        for _ in range(K):
            fns[name]()
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    graph = e0.elapsed_time(e1) / K * 1e3
    print("%-22s n=%d  %.2f us/launch plain  %.2f us/launch in a graph" % (name, n, plain, graph))
