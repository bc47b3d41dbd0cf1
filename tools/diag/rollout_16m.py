"""Three 16,777,216-game random rollouts (PMC target for the issue-rate check)."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import ops  # noqa: E402

n = 1 << 24
h = torch.zeros(133, dtype=torch.int64, device="cuda")
ops.rollout(n, 1, 0, hist=h, device="cuda", want_boards=False, want_diff=False, want_plies=False)
torch.cuda.synchronize()
h.zero_()
t0 = time.perf_counter()
for k in range(3):
    ops.rollout(n, 1, (k + 1) * n, hist=h, device="cuda", want_boards=False, want_diff=False, want_plies=False)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print("16M x3: %.3f ms/launch, %.3e env-steps/s" % (dt / 3 * 1e3, int(h[132]) / dt))
