"""The C-ABI from a plain C++ host (examples/rollout_host.cpp): built with
hipcc against include/othello.h and the in-tree library, run as its own
process, output checked against the oracle."""
import os
import re
import subprocess

import pytest

import oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_host_example(tmp_path):
    exe = str(tmp_path / "rollout_host")
    lib = os.path.join(ROOT, "subproc_amd", "lib")
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O2", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "examples", "rollout_host.cpp"), "-L" + lib, "-lsubproc_amd_hip",
                           "-Wl,-rpath," + lib, "-o", exe])
    n = 4096
    out = subprocess.run([exe, str(n)], capture_output=True, text=True, timeout=120, check=True).stdout
    o = oracle.rollout(n, 0x5EED, 0, n_random=0)
    h = o["hist"]
    m = re.search(r"games (\d+) black (\d+) white (\d+) draws (\d+) env-steps (\d+)", out)
    assert [int(x) for x in m.groups()] == [n, int(h[129]), int(h[130]), int(h[131]), int(h[132])]
    fb = re.search(r"game0 final black ([0-9a-f]+) white ([0-9a-f]+)", out)
    assert int(fb.group(1), 16) == int(o["final_boards"][0, 0]) and int(fb.group(2), 16) == int(o["final_boards"][0, 1])
    assert "step d3 ret 1" in out
