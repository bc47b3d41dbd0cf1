"""Twenty single-stream 1,048,576-game random rollouts after a 300 ms warm-up
(PMC / kernel-trace target for per-launch counts of the headline kernel)."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from subproc_amd import ops  # noqa: E402

n = 1 << 20
h = torch.zeros(133, dtype=torch.int64, device="cuda")
t_end = time.perf_counter() + 0.3
k = 0
while time.perf_counter() < t_end:
    ops.rollout(n, 1, k * n, hist=h, device="cuda", want_boards=False, want_diff=False, want_plies=False)
    torch.cuda.synchronize()
    k += 1
h.zero_()
t0 = time.perf_counter()
for j in range(20):
    ops.rollout(n, 1, (k + j) * n, hist=h, device="cuda", want_boards=False, want_diff=False, want_plies=False)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print("1M x20: %.4f ms/launch, %.4e env-steps/s" % (dt / 20 * 1e3, int(h[132]) / dt))
