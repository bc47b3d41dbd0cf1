"""The VGPR-bank pass (tools/vgpr_banks.py, a round-3 experiment that builds the
A/B libraries of tools/diag/r03_banks*.sh): a consistent renaming of register
pairs that lowers the hot loop's three-source same-bank v_bitop3_b32 count and
leaves every tuple whole.  CPU only: it works on gfx950 assembly text (the
round-3 GPU suite ran green on a library with every kernel renamed)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import vgpr_banks as vb  # noqa: E402

KERNEL = """\
_Zdemo:
\tv_mov_b32_e32 v2, v0
\tglobal_load_dwordx4 v[4:7], v[2:3], off
\tds_read2st64_b64 v[8:11], v2 offset1:1
.LBB0_1:                                ; =>This Inner Loop Header: Depth=1
\tv_bitop3_b32 v12, v16, v20, v24 bitop3:0xca
\tv_bitop3_b32 v13, v17, v21, v25 bitop3:0xca
\tv_bitop3_b32 v14, v4, v8, v12 bitop3:0x80
\tv_bitop3_b32 v15, v5, v9, v13 bitop3:0x80
\tv_lshlrev_b64 v[16:17], 7, v[12:13]
\tv_bitop3_b32 v18, v28, v24, v16 bitop3:0xfe
\ts_cbranch_scc1 .LBB0_1
; %bb.2:
\tglobal_store_dwordx4 v[2:3], v[4:7], off
\ts_endpgm
.Lfunc_end0:
\t.amdhsa_kernel _Zdemo
\t\t.amdhsa_next_free_vgpr 29
\t\t.amdhsa_accum_offset 32
\t.end_amdhsa_kernel
"""


def _conflicts(lines, lo, hi):
    idx = vb.hot_loop_lines(lines, lo, hi) or range(lo, hi)  # a kernel without a loop: its body
    return vb.conflicts(vb.triples(lines, idx), {p: p & 1 for p in range(128)})


def _regs(line):
    out = []
    for m in vb.REG.finditer(vb.code(line)):
        if m.group(1) is not None:
            out.append((int(m.group(1)),))
        else:
            out.append(tuple(range(int(m.group(2)), int(m.group(3)) + 1)))
    return out


def _check_renaming(before, after, lo, hi):
    """a consistent pair renaming: one map for the whole kernel, a bijection,
    halves kept, tuples consecutive and even-aligned, v0 in place"""
    mp = {}
    for x, y in zip(before[lo:hi], after[lo:hi]):
        if x.lstrip().startswith("."):  # labels and directives (a descriptor may sit inside the range)
            continue
        rx, ry = _regs(x), _regs(y)
        assert len(rx) == len(ry), (x, y)
        assert re.sub(vb.REG, "R", vb.code(x)).rstrip() == re.sub(vb.REG, "R", vb.code(y)).rstrip()
        for a, b in zip(rx, ry):
            assert len(a) == len(b)
            if len(b) > 1:
                assert b[0] % 2 == 0 and list(b) == list(range(b[0], b[0] + len(b)))
            for r, s in zip(a, b):
                assert mp.setdefault(r, s) == s, "register %d renamed two ways" % r
    assert len(set(mp.values())) == len(mp)
    assert all(r % 2 == s % 2 for r, s in mp.items())
    assert all(mp[r] // 2 == mp[r ^ 1] // 2 for r in mp if r ^ 1 in mp)
    assert mp.get(0, 0) == 0


def test_demo_kernel():
    lines = KERNEL.split("\n")
    (name, lo, hi), = vb.functions(lines)
    before = list(lines)
    c0 = _conflicts(lines, lo, hi)
    assert c0 == 5  # pairs (8, 10, 12) and (2, 4, 6) in both halves, (14, 12, 8) once: all even
    b, a = vb.permute_function(lines, lo, hi, name)
    assert (b, a) == (c0, _conflicts(lines, lo, hi))
    assert a < b
    _check_renaming(before, lines, lo, hi)


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc")
def test_othello_kernels(tmp_path):
    """the real kernels: every renaming consistent, the headline loop's conflicts
    not above hipcc's, and no kernel's VGPR count above its reserved budget"""
    s = tmp_path / "othello.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    "--cuda-device-only", "-S", "-o", str(s), os.path.join(ROOT, "subproc_amd", "csrc", "othello.hip")],
                   check=True, capture_output=True)
    lines = s.read_text().split("\n")
    before = list(lines)
    seen = 0
    for name, lo, hi in vb.functions(lines):
        c0 = _conflicts(lines, lo, hi)
        d = vb.descriptor(lines, name)
        free0 = int(lines[d["next_free"]].split()[-1])
        b, a = vb.permute_function(lines, lo, hi, name)
        assert a <= b == c0
        _check_renaming(before, lines, lo, hi)
        free1 = int(lines[d["next_free"]].split()[-1])
        assert free1 == free0 or free0 < free1 <= int(lines[d["accum"]].split()[-1])
        if "rollout_kernelILi0ELb0ELb0E" in name:
            # the headline loop: the pass leaves at most half of hipcc's
            # same-bank triples (round 5, with the batch-tail hand-over in
            # the two-ply loop: 14 -> 4; round 4: 2 -> 0)
            assert a <= max(2, b // 2), (b, a)
            seen += 1
    assert seen == 1
