#!/usr/bin/env python3
"""Diagnostic (NOT product build): rewrite the VOP1/VOP2 (_e32) VALU
instructions of hipcc's gfx950 assembly into their VOP3 (_e64) encodings.

tools/diag/valu_rate7.cpp measured on the box that a fast instruction issued
after a slow VOP3 one (64-bit shift, v_lshl_add_u64, v_bcnt) costs ~2.9
cycles in its VOP3 encoding (v_bitop3_b32, v_and_b32_e64) against ~3.6 in its
VOP2 one (v_and_b32_e32), and that a slow VOP1 (v_bfrev_b32_e32) in front
loses the gain.  This pass tests the effect on the real kernels.

Left alone: instructions with a literal (gfx9 VOP3 takes no literal), and
those whose e64 form would read the constant bus twice (an SGPR source
beside an implicit VCC read).
    python tools/diag/vop3_promote.py in.s out.s [name-substring ...] [--only=op1,op2]
(--only: promote just these mnemonics, e.g. v_min_u32,v_cndmask_b32)
"""
import re
import sys

INLINE = re.compile(r"^-?(\d+)$")


def literal(tok):
    tok = tok.strip()
    if tok.startswith("0x") or tok.startswith("-0x"):
        v = int(tok, 16)
        return not (-16 <= v <= 64)
    m = INLINE.match(tok)
    if m:
        return not (-16 <= int(tok) <= 64)
    return False


def sgpr(tok):
    tok = tok.strip()
    return tok.startswith("s") or tok in ("vcc", "vcc_lo", "vcc_hi", "exec", "exec_lo", "exec_hi", "m0")


def promote(line, only=None):
    m = re.match(r"^(\s+)(v_\w+)_e32(\s+)(.*)$", line)
    if not m:
        return line, False
    ind, op, sp, rest = m.groups()
    if only and op not in only:
        return line, False
    ops = [t.strip() for t in rest.split(";")[0].split(",")]
    if any(literal(t) for t in ops):
        return line, False
    if op.startswith("v_readfirstlane") or op.startswith("v_nop") or "dpp" in rest or "sdwa" in rest:
        return line, False
    # implicit VCC reads: v_cndmask (src2 vcc), v_addc/subb (carry-in)
    reads_vcc = op.startswith("v_cndmask") or op.startswith("v_addc") or op.startswith("v_subb")
    if reads_vcc and any(sgpr(t) for t in ops[1:-1] if t != "vcc"):
        return line, False
    if (op.startswith("v_cmp") or op.startswith("v_cmpx")) and not (only and op in only):
        return line, False  # e32 writes vcc implicitly; keep hipcc's choice
    return "%s%s_e64%s%s" % (ind, op, sp, rest), True


def main():
    src, dst = sys.argv[1], sys.argv[2]
    only = [a.split("=", 1)[1].split(",") for a in sys.argv[3:] if a.startswith("--only=")]
    only = set(only[0]) if only else None
    pats = [a for a in sys.argv[3:] if not a.startswith("--")] or ["_Z"]
    lines = open(src).read().split("\n")
    cur, n = None, 0
    for i, ln in enumerate(lines):
        fm = re.match(r"^(_Z\w+):", ln)
        if fm:
            cur = fm.group(1)
        elif ln.strip().startswith(".Lfunc_end"):
            cur = None
        if cur and any(p in cur for p in pats):
            lines[i], ch = promote(ln, only)
            n += ch
    open(dst, "w").write("\n".join(lines))
    print("vop3_promote: %d instructions promoted" % n)


if __name__ == "__main__":
    main()
