"""Every committed fixture regenerates from the reference, byte for byte.

tests/golden/gen_golden.py drives the reference itself (board.py through its
two-line shim, parameter_progress_position_moves_learn.py, learn_base.py and
progress_position_moves_learn.py exec'd against stubs of their network
imports) and writes the 24 fixtures the parity tests read.  This test runs it
into a temp dir with one command and compares every file with the committed
one.  It needs /root/reference, so it only runs in the build container (the
GPU box has no reference; it is skipped there).
"""
import filecmp
import os
import subprocess
import sys

import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REFERENCE = "/root/reference/board.py"


def committed_fixtures():
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith((".json", ".npz")))


def test_fixture_count():
    assert len(committed_fixtures()) == 24, committed_fixtures()


@pytest.mark.skipif(not os.path.exists(REFERENCE), reason="needs /root/reference (build container only)")
@pytest.mark.timeout(900)
def test_all_fixtures_regenerate_byte_identical(tmp_path):
    out = tmp_path / "golden"
    subprocess.run([sys.executable, os.path.join(GOLDEN, "gen_golden.py"), "--out", str(out)], check=True,
                   stdout=subprocess.DEVNULL, timeout=840)
    written = sorted(f for f in os.listdir(out) if f.endswith((".json", ".npz")))
    assert written == committed_fixtures()
    differ = [f for f in written if not filecmp.cmp(os.path.join(GOLDEN, f), os.path.join(out, f), shallow=False)]
    assert not differ, "fixtures that no longer match the reference's output: %s" % differ
