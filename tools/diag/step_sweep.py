"""Step-kernel timing (config 2 steady state, 16M boards) — run on the GPU box.

  python tools/diag/step_sweep.py [LIB.so] [--no-legal]
LIB defaults to the product library; diagnostic builds of kernel variants can be
passed instead (same C-ABI)."""
import ctypes
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import _lib, ops  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
path = args[0] if args else _lib.LIB_PATH
lib = ctypes.CDLL(path)
res, argt = _lib.SIGNATURES["oth_step"]
lib.oth_step.restype, lib.oth_step.argtypes = res, argt
want_legal = "--no-legal" not in sys.argv

n = 1 << 24
pos = ops.sample_midgame(n, 0x5EED, device="cuda")
outs = [torch.empty_like(pos.boards), torch.empty_like(pos.turn), torch.empty(n, dtype=torch.int64, device="cuda"),
        torch.empty(n, dtype=torch.int64, device="cuda"), torch.empty(n, dtype=torch.int8, device="cuda")]
s = torch.cuda.current_stream()
args = (pos.boards.data_ptr(), pos.turn.data_ptr(), pos.move.data_ptr(), outs[0].data_ptr(), outs[1].data_ptr(),
        outs[2].data_ptr(), outs[3].data_ptr() if want_legal else None, outs[4].data_ptr(), None, n, s.cuda_stream)
for _ in range(5):
    assert lib.oth_step(*args) == 0
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    lib.oth_step(*args)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
nb = 52 if want_legal else 44
print("%s legal=%d bpc=%s %.1f us  %.2f TB/s" % (os.path.basename(path), want_legal,
      os.environ.get("OTH_STEP_BLOCKS_PER_CU", "-"), us, n * nb / us / 1e6))
