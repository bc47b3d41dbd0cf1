#!/usr/bin/env python3
"""Static VALU instruction mix of each kernel's hot loop -> the issue ceiling
bench.py prices the integer kernels against (profiles/valu_mix.json).

CDNA4 SIMDs are 32 lanes wide: a wave64 VALU instruction can issue every 2
cycles (MI355X_MICROARCH.md, cycle constants).  Measured on the box
(tools/diag/valu_rate5.cpp, DESIGN.md §3 cost model), only bitwise logic and
moves stream at ~2.2 cycles and v_bitop3_b32 at ~2.5 (4.3 with its three
sources in one VGPR bank); shifts, bit reversal, popcount, selects, compares,
multiplies and even 32-bit add/sub/min take 4.1-4.4.  So a kernel's ceiling is
1024 SIMDs x clock / (mean cycles over its mix).
The hot loop is the innermost LLVM loop (its header and every block tagged
"in Loop: Header=<it>") holding the most VALU instructions; counts are static
(every block once), so rarely-taken blocks inside the loop are included.
    python tools/valu_mix.py [--asm file.s] > profiles/valu_mix.json
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# Measured on the box (tools/diag/valu_rate5.cpp: 32 independent instructions
# on fixed registers, 8 waves/SIMD): bitwise logic, moves, 32-bit add/sub
# without carry and the 16-bit VOP2 ops stream at ~2.2 cycles per
# wave-instruction; v_bitop3_b32 at 2.5 -- 4.3 when its three source registers
# are distinct and in one VGPR bank (bank = number mod 4); every shift,
# min/max, compare, carry, select, popcount and 64-bit op at 4.0-4.4.
FAST = re.compile(r"^v_((and|or|xor|not|mov)_b32|(add|sub)_u32|(lshlrev|lshrrev)_b16|(add|sub|min)_u16|mul_lo_u16)(_e32)?$")
FAST_CYC, SLOW_CYC = 2.2, 4.2
BITOP3_CYC, BITOP3_CONFLICT_CYC = 2.5, 4.3
MEASURED = {"v_lshlrev_b64": 4.25, "v_lshrrev_b64": 4.22, "v_lshl_add_u64": 4.24, "v_bfrev_b32_e32": 4.13,
            "v_lshlrev_b32_e32": 4.07, "v_bcnt_u32_b32": 4.09, "v_mul_hi_u32": 4.29, "v_mad_u64_u32": 4.43,
            "v_cndmask_b32_e64": 4.2, "v_bfe_u32": 4.25, "v_min_u32_e32": 4.08, "v_sub_u32_e32": 4.08,
            "v_bfi_b32": 4.2, "v_or3_b32": 4.2, "v_alignbit_b32": 4.12, "v_perm_b32": 4.2,
            # round 3 (valu_rate5.cpp OPs 24-57)
            "v_add_u32_e32": 2.19, "v_sub_u32_e32": 2.24, "v_min_u32_e32": 4.06, "v_max_u32_e32": 4.05,
            "v_add_co_u32_e32": 4.09, "v_sub_co_u32_e32": 4.09, "v_sub_co_u32_e64": 4.09, "v_addc_co_u32_e32": 4.09,
            "v_cmp_gt_u32_e32": 4.03, "v_cndmask_b32_e32": 4.0, "v_add3_u32": 4.13, "v_lshl_or_b32": 4.10,
            "v_and_or_b32": 4.11, "v_mov_b64_e32": 4.14, "v_ffbh_u32_e32": 4.05, "v_bfe_u32": 4.20}


# Costs inside a mixed loop (tools/diag/valu_rate7.cpp, 8 waves/SIMD, slow
# VOP3 instructions interleaved with fast ones): a fast instruction costs ~2.95
# cycles in a VOP3 encoding (v_bitop3_b32, v_and/or_b32_e64) and ~3.7 in a
# VOP1/VOP2 one (v_and_b32_e32 ...), against 2.2-2.5 when streamed alone; the
# slow ones keep their isolated cost.  "mean_cycles_mixed" prices a loop so.
MIXED_FAST_VOP3, MIXED_FAST_E32 = 2.95, 3.7


def cycles_mixed(op, line=None):
    if op == "v_bitop3_b32":
        return BITOP3_CONFLICT_CYC if bank_conflict(line) else MIXED_FAST_VOP3
    c = cycles(op, line)
    if c < 3.0:  # a fast instruction
        return MIXED_FAST_VOP3 if op.endswith("_e64") else MIXED_FAST_E32
    return c


def bank_conflict(line):
    """three distinct source VGPRs in one bank (v_bitop3_b32 vD, vA, vB, vC)"""
    m = re.match(r"\s*v_bitop3_b32\s+v\d+,\s*v(\d+),\s*v(\d+),\s*v(\d+)", line or "")
    if not m:
        return False
    regs = {int(g) for g in m.groups()}
    return len(regs) == 3 and len({r % 4 for r in regs}) == 1


def cycles(op, line=None):
    if op == "v_bitop3_b32":
        return BITOP3_CONFLICT_CYC if bank_conflict(line) else BITOP3_CYC
    if op in MEASURED:
        return MEASURED[op]
    return FAST_CYC if FAST.match(op) else SLOW_CYC
KERNELS = {"rollout_kernel<0, false>": "rollout_kernelILi0ELb0ELb0E", "rollout_kernel<1, false>": "rollout_kernelILi1ELb0ELb0E",
           "rollout_kernel<2, false>": "rollout_kernelILi2ELb0ELb0E", "step_kernel": "step_kernel"}


def compile_asm():
    out = os.path.join(tempfile.mkdtemp(), "othello.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-mllvm", "-pragma-unroll-threshold=200000",
                    "-x", "hip", "--cuda-device-only", "-S",
                    "-o", out, os.path.join(ROOT, "subproc_amd", "csrc", "othello.hip"),
                    "-I", os.path.join(ROOT, "include")], check=True, capture_output=True)
    return out


def functions(lines):
    cur, body = None, []
    for ln in lines:
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            body.append(ln)
            if ln.startswith("\t.size\t" + cur) or ln.strip().startswith(".Lfunc_end"):
                yield cur, body
                cur = None
    if cur:
        yield cur, body


def hot_loop_mix(body):
    blocks, order, label = collections.defaultdict(list), [], None
    header_of = {}
    for ln in body:
        m = re.match(r"^\.(LBB\w+):(.*)", ln)
        if m:
            label = m.group(1)
            order.append(label)
            h = re.search(r"Header=(BB\w+)", m.group(2))
            if h:
                header_of[label] = "L" + h.group(1)
            if "Inner Loop Header" in m.group(2):
                header_of[label] = label
            continue
        if label and re.match(r"^\s+; =>\s*This Inner Loop Header", ln):  # the comment on its own line
            header_of[label] = label
            continue
        m = re.match(r"^\s+(v_[a-z0-9_]+)", ln)
        if m and label:
            blocks[label].append((m.group(1), ln))
    loops = collections.defaultdict(list)
    for b, h in header_of.items():
        loops[h].extend(blocks[b])
    inner = {h: ops for h, ops in loops.items() if header_of.get(h) == h}
    if not inner:
        return None
    h, ops = max(inner.items(), key=lambda kv: len(kv[1]))
    return mix_of(ops, h)


def mix_of(ops, header):
    names = [o for o, _ in ops]
    fast = sum(1 for o in names if FAST.match(o))
    mean = sum(cycles(o, ln) for o, ln in ops) / max(1, len(ops))
    mixed = sum(cycles_mixed(o, ln) for o, ln in ops) / max(1, len(ops))
    return {"loop_header": header, "valu": len(ops), "fast_vop2": fast, "slow": len(ops) - fast,
            "bitop3_bank_conflicts": sum(1 for o, ln in ops if o == "v_bitop3_b32" and bank_conflict(ln)),
            "e32_fast": sum(1 for o, ln in ops if o.endswith("_e32") and cycles(o, ln) < 3.0),
            "mean_cycles": round(mean, 3), "mean_cycles_mixed": round(mixed, 3),
            "top": collections.Counter(names).most_common(8)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--asm")
    a = p.parse_args()
    path = a.asm or compile_asm()
    lines = open(path).read().splitlines()
    out = {"fast_cycles": FAST_CYC, "slow_cycles": SLOW_CYC, "simds": 1024, "clock_ghz": 2.4, "kernels": {}}
    for name, body in functions(lines):
        for k, pat in KERNELS.items():
            if pat in name:
                r = hot_loop_mix(body)
                if r is None:  # no loop (elementwise kernels): the whole body
                    ops = [(m.group(1), ln) for m, ln in ((re.match(r"^\s+(v_[a-z0-9_]+)", ln), ln) for ln in body) if m]
                    r = mix_of(ops, None)
                r["peak_winstr_s"] = out["simds"] * out["clock_ghz"] * 1e9 / r["mean_cycles"]
                r["peak_winstr_s_mixed"] = out["simds"] * out["clock_ghz"] * 1e9 / r["mean_cycles_mixed"]
                if k == "rollout_kernel<0, false>":
                    r["plies_per_loop_iteration"] = 2  # round 3: the random loop body is two plies
                out["kernels"][k] = r
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
