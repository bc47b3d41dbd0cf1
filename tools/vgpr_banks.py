#!/usr/bin/env python3
"""Re-number a kernel's VGPR pairs so that its hot loop's v_bitop3_b32
instructions do not read three registers of one VGPR bank (round-3
experiment; measured, not part of the shipped build:
profiles/design_history_r01_r04.md §3, "VGPR banks").

Why: a v_bitop3_b32 whose three source registers are distinct and sit in one
bank (register number mod 4) issued in 4.3 cycles instead of 2.5 in the
cost-model probe (tools/diag/valu_rate5.cpp), and hipcc's allocation decides
that: the only handle HIP source has on it is the order the code is written
in, a lottery small source changes lose (the batch-tail hand-over moved the
random rollout's loop from 2 to 12 such instructions).  A consistent renaming of
physical registers changes nothing a kernel computes, so this pass renames
them after the fact, on hipcc's gfx950 assembly.

The renaming permutes aligned register PAIRS (v[2k:2k+1] -> v[2j:2j+1], halves
kept in order): every 64-bit operand stays an aligned pair, and the bank of a
register becomes 2 * (j mod 2) + (its half).  Three same-half sources from three
pairs conflict iff the three target pair indices have one parity, so the choice
is a two-colouring of the pairs with as many of each parity as there are slots.
Pairs linked by a wider tuple (v[a:a+3] of a 128-bit load) move as one block to
consecutive slots; the pair holding v0 (the work-item ids at entry) and
odd-aligned tuples stay.  A local search minimises the conflicting triples,
weighted by loop depth (the hot loop most).  Slots run up to the kernel's
accumulation offset, so the register budget does not change.

    python tools/vgpr_banks.py in.s out.s KERNEL_SYMBOL_SUBSTRING [...]
        rewrite hipcc's device assembly (prints conflicts before -> after)
    python tools/vgpr_banks.py --build-lib OUT.so [SRC.hip]
        the HIP library with the pass applied to every kernel of SRC
        (default subproc_amd/csrc/othello.hip): hipcc's own steps (device
        assembly, assemble, link, bundle, host compile against the bundle)
        with this pass between the first two -- the A/B builds of
        tools/diag/r03_banks*.sh
"""
import random
import re
import sys

REG = re.compile(r"(?<![\w.\[])v(?:(\d+)|\[(\d+):(\d+)\])(?![\w\]])")
BITOP3 = re.compile(r"^\s*v_bitop3_b32\s+v\d+,\s*v(\d+),\s*v(\d+),\s*v(\d+)\b")


def functions(lines):
    """(name, first body line index, end index) of each kernel symbol"""
    out, cur, start = [], None, 0
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\w+):", ln)
        if m:
            cur, start = m.group(1), i + 1
            continue
        if cur and (ln.strip().startswith(".Lfunc_end") or ln.startswith("\t.size\t" + cur)):
            out.append((cur, start, i))
            cur = None
    return out


def code(ln):
    return ln.split(";", 1)[0]


def hot_loop_lines(lines, lo, hi):
    """line indices of the innermost loop with the most VALU (hipcc's loop comments)"""
    header_of, label, blocks = {}, None, {}
    for i in range(lo, hi):
        ln = lines[i]
        m = re.match(r"^\.(LBB\w+):(.*)", ln)
        if m:
            label = m.group(1)
            blocks[label] = []
            h = re.search(r"Header=(BB\w+)", m.group(2))
            if h:
                header_of[label] = "L" + h.group(1)
            if "Inner Loop Header" in m.group(2):
                header_of[label] = label
            continue
        if label and re.match(r"^\s+; =>\s*This Inner Loop Header", ln):
            header_of[label] = label
            continue
        if label:
            blocks[label].append(i)
    loops = {}
    for b, h in header_of.items():
        loops.setdefault(h, []).extend(blocks[b])
    inner = {h: idx for h, idx in loops.items() if header_of.get(h) == h}
    if not inner:
        return []
    return max(inner.values(), key=lambda idx: sum(1 for i in idx if re.match(r"^\s+v_", lines[i])))


def loop_depths(lines, lo, hi):
    """{line index: loop depth} from hipcc's block comments (0 outside loops)"""
    out, depth = {}, 0
    for i in range(lo, hi):
        ln = lines[i]
        m = re.match(r"^\.(LBB\w+):(.*)", ln)
        if m:
            d = re.search(r"Depth=(\d+)", m.group(2))
            depth = int(d.group(1)) if d else 0
            continue
        if re.match(r"^\s+; =>\s*This Inner Loop Header: Depth=(\d+)", ln):
            depth = int(re.search(r"Depth=(\d+)", ln).group(1))
            continue
        out[i] = depth
    return out


def weighted_triples(lines, lo, hi):
    """every same-half triple of the kernel, weighted: the hot loop's count
    most, then by loop depth (a block at depth d runs ~8^d times as often)"""
    hot = set(hot_loop_lines(lines, lo, hi))
    depth = loop_depths(lines, lo, hi)
    out = []
    for i in range(lo, hi):
        t = triples(lines, [i])
        if t:
            w = 4096 if i in hot else 8 ** depth.get(i, 0)
            out.append((t[0], w))
    return out


def triples(lines, idx):
    out = []
    for i in idx:
        m = BITOP3.match(code(lines[i]))
        if m:
            r = [int(g) for g in m.groups()]
            if len(set(r)) == 3 and len({x & 1 for x in r}) == 1:  # same half: a bank collision is possible
                out.append(tuple(x >> 1 for x in r))
    return out


def conflicts(trip, colour):
    return sum(1 for a, b, c in trip if colour[a] == colour[b] == colour[c])


def solve(trip, npairs, chains, pinned, seed=1, restarts=24, steps=3000, weights=None):
    """slot of every pair (a permutation of 0..npairs-1) minimising the triples
    whose three pairs land on slots of one parity.  chains: intervals of pairs
    (tuple-linked, lo..hi) that move as one block to consecutive slots; pinned:
    chains that stay.  Starts from the identity; returns (slot, cost)."""
    rng = random.Random(seed)
    chain_of = {}
    for c in chains:
        for p in range(c[0], c[1] + 1):
            chain_of[p] = c
    single = [p for p in range(npairs) if p not in chain_of]
    movable_chains = [c for c in chains if c not in pinned]

    w = weights or [1] * len(trip)
    touch = {}
    for k, t in enumerate(trip):
        for p in set(t):
            touch.setdefault(p, []).append(k)

    def hit(slot, k):
        a, b, c = trip[k]
        return w[k] if (slot[a] & 1) == (slot[b] & 1) == (slot[c] & 1) else 0

    def cost(slot):
        return sum(hit(slot, k) for k in range(len(trip)))

    ident = list(range(npairs))
    best, best_cost = ident[:], cost(ident)
    for restart in range(restarts):
        slot = ident[:]
        if restart:  # a random start: shuffle the single pairs among their slots
            sl = [slot[p] for p in single]
            rng.shuffle(sl)
            for p, q in zip(single, sl):
                slot[p] = q
        cur = cost(slot)
        for _ in range(steps):
            if cur == 0:
                break
            moved = {}  # pair -> new slot
            if movable_chains and rng.random() < 0.2:
                c = rng.choice(movable_chains)
                L = c[1] - c[0] + 1
                s0 = slot[c[0]]
                t = rng.randrange(0, npairs - L + 1)
                if abs(t - s0) < L:
                    continue
                occupant = {slot[p]: p for p in range(npairs)}
                region = [occupant[t + k] for k in range(L)]
                if any(q in chain_of for q in region):
                    continue
                for k in range(L):
                    moved[c[0] + k] = t + k
                    moved[region[k]] = s0 + k
            else:
                a, b = rng.sample(single, 2)
                if (slot[a] & 1) == (slot[b] & 1):
                    continue
                moved[a], moved[b] = slot[b], slot[a]
            ks = {k for p in moved for k in touch.get(p, ())}
            old = {p: slot[p] for p in moved}
            before = sum(hit(slot, k) for k in ks)
            for p, q in moved.items():
                slot[p] = q
            delta = sum(hit(slot, k) for k in ks) - before
            if delta <= 0 or rng.random() < 0.01:
                cur += delta
                if cur < best_cost:
                    best, best_cost = slot[:], cur
            else:
                for p, q in old.items():
                    slot[p] = q
        if best_cost == 0:
            break
    return best, best_cost


def descriptors(lines):
    """{kernel: line indices of its .amdhsa_next_free_vgpr / .amdhsa_accum_offset,
    its metadata .vgpr_count and its '.set NAME.num_vgpr'} in one pass"""
    out, cur, entry = {}, None, None
    for i, ln in enumerate(lines):
        t = ln.strip()
        if t.startswith(".amdhsa_kernel "):
            cur = t.split()[1]
        elif cur and t.startswith(".amdhsa_next_free_vgpr"):
            out.setdefault(cur, {})["next_free"] = i
        elif cur and t.startswith(".amdhsa_accum_offset"):
            out.setdefault(cur, {})["accum"] = i
        elif t.startswith(".end_amdhsa_kernel"):
            cur = None
        elif t.startswith(".set ") and t.split()[1].endswith(".num_vgpr,"):
            out.setdefault(t.split()[1][: -len(".num_vgpr,")], {})["set"] = i
        elif t.startswith("- .agpr_count:") or t == "-":
            entry = []  # a new metadata map (kernels are list entries)
        if entry is not None:
            if t.startswith(".name:"):
                entry.append(("name", t.split()[-1]))
            elif t.startswith(".vgpr_count:"):
                entry.append(("meta", i))
            names = [v for k, v in entry if k == "name"]
            metas = [v for k, v in entry if k == "meta"]
            if names and metas:
                out.setdefault(names[0], {})["meta"] = metas[0]
    return out


def descriptor(lines, name):
    return descriptors(lines).get(name, {})


def permute_function(lines, lo, hi, name=None, desc=None):
    regs_used, links, pinned_pairs = set(), set(), {0}  # pair 0 holds v0 (work-item ids) at entry
    for i in range(lo, hi):
        c = code(lines[i])
        if re.search(r"(?<![\w.])a\[?\d", c) and re.match(r"^\s+(v_accvgpr|v_mfma)", c):
            raise SystemExit("vgpr_banks: AGPR code is not handled")
        if re.match(r"^\s+s_(swappc|setpc|call)", c):
            raise SystemExit("vgpr_banks: calls are not handled")
        for m in REG.finditer(c):
            if m.group(1) is not None:
                regs_used.add(int(m.group(1)))
                continue
            a, b = int(m.group(2)), int(m.group(3))
            regs_used.update(range(a, b + 1))
            if a % 2:  # an odd-aligned tuple: leave its registers alone
                pinned_pairs.update(range(a >> 1, (b >> 1) + 1))
            else:  # v[a:b] spans pairs a/2 .. b/2, which must stay consecutive
                links.update(range(a >> 1, b >> 1))  # p linked to p + 1
    if not regs_used:
        return 0, 0
    n = max(regs_used) + 1
    # slots: every pair below the kernel's accumulation offset (the VGPRs its
    # descriptor reserves, n rounded up to 4), so the renaming may use a pair
    # the allocation left free without changing the kernel's register budget
    if desc is None:
        desc = descriptor(lines, name) if name else {}
    limit = n
    if "accum" in desc and "next_free" in desc and int(lines[desc["next_free"]].split()[-1]) == n:
        # (a kernel with AGPRs counts them in next_free_vgpr: no slack taken there)
        limit = max(n, int(lines[desc["accum"]].split()[-1]))
    npairs = limit // 2  # a trailing half-used pair stays where it is
    # chains: maximal runs of linked pairs; single pairs are not chains
    chains, p = [], 0
    while p < npairs:
        q = p
        while q in links and q + 1 < npairs:
            q += 1
        if q > p or p in pinned_pairs:
            chains.append((p, q))
        p = q + 1
    pinned = {c for c in chains if any(x in pinned_pairs for x in range(c[0], c[1] + 1))}
    pinned |= {c for c in chains if c[1] + 1 in links}  # runs into the trailing pair
    hot = [t for t in triples(lines, hot_loop_lines(lines, lo, hi) or range(lo, hi)) if max(t) < npairs]
    before = conflicts(hot, {x: x & 1 for x in range(npairs)})
    wt = [(t, w) for t, w in weighted_triples(lines, lo, hi) if max(t) < npairs]
    trip, weights = [t for t, _ in wt], [w for _, w in wt]
    ident_cost = sum(w for (a, b, c), w in wt if (a & 1) == (b & 1) == (c & 1))
    if ident_cost == 0:
        return before, before
    slot, cost = solve(trip, npairs, chains, pinned, weights=weights)
    if cost >= ident_cost:
        return before, before
    assert sorted(slot) == list(range(npairs))
    perm = {x: slot[x] for x in range(npairs)}
    perm.update({x: x for x in range(npairs, (limit + 1) // 2)})

    def reg(r):
        return 2 * perm[r >> 1] + (r & 1)

    def sub(m):
        if m.group(1) is not None:
            return "v%d" % reg(int(m.group(1)))
        a, b = int(m.group(2)), int(m.group(3))
        # a tuple's pairs were moved as one block: still consecutive, still aligned
        assert all(reg(r) == reg(a) + (r - a) for r in range(a, b + 1)), "tuple v[%d:%d] split" % (a, b)
        assert reg(a) % 2 == a % 2
        return "v[%d:%d]" % (reg(a), reg(a) + (b - a))

    for i in range(lo, hi):
        c = code(lines[i])
        if "v" in c and not c.lstrip().startswith("."):
            lines[i] = REG.sub(sub, c).rstrip()
    new_n = max(reg(r) for r in regs_used) + 1
    if new_n > n:  # a pair moved into the reserved slack: the counts say so
        assert "next_free" in desc and "meta" in desc and new_n <= limit, "no descriptor to update"
        for key in ("next_free", "meta", "set"):
            if key in desc:
                ln = lines[desc[key]]
                lines[desc[key]] = ln[: ln.rstrip().rfind(" ") + 1] + str(new_n)
    trip2 = triples(lines, hot_loop_lines(lines, lo, hi) or range(lo, hi))
    return before, conflicts(trip2, {x: x & 1 for x in range((limit + 1) // 2)})


def build_library(out_so, src=None):
    import os
    import subprocess
    import tempfile

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = src or os.path.join(root, "subproc_amd", "csrc", "othello.hip")
    hipcc, llvm = "/opt/rocm/bin/hipcc", "/opt/rocm/lib/llvm/bin"
    inc = ["-I", os.path.join(root, "include")]
    with tempfile.TemporaryDirectory() as tmp:
        j = lambda f: os.path.join(tmp, f)  # noqa: E731
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", *inc, "--cuda-device-only", "-S",
                               "-o", j("o.s"), src], stderr=subprocess.DEVNULL)
        subprocess.check_call([sys.executable, os.path.abspath(__file__), j("o.s"), j("b.s"), "_Z"])
        subprocess.check_call([os.path.join(llvm, "clang"), "-x", "assembler", "-target", "amdgcn-amd-amdhsa",
                               "-mcpu=gfx950", "-c", "-o", j("dev.o"), j("b.s")])
        subprocess.check_call([os.path.join(llvm, "ld.lld"), "-shared", "-o", j("o.hsaco"), j("dev.o")])
        subprocess.check_call([os.path.join(llvm, "clang-offload-bundler"), "-type=o", "-bundle-align=4096",
                               "-targets=host-x86_64-unknown-linux-gnu,hipv4-amdgcn-amd-amdhsa--gfx950",
                               "-input=/dev/null", "-input=" + j("o.hsaco"), "-output=" + j("o.hipfb")])
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *inc, "--cuda-host-only",
                               "-Xclang", "-fcuda-include-gpubinary", "-Xclang", j("o.hipfb"), "-c", "-o", j("oth.o"),
                               src])
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *inc, "-c",
                               "-o", j("td.o"), os.path.join(root, "subproc_amd", "csrc", "td_table.hip")])
        subprocess.check_call([hipcc, "--offload-arch=gfx950", "-fPIC", "-shared",
                               "-Wl,--version-script=" + os.path.join(root, "subproc_amd", "csrc", "exports.map"),
                               "-o", out_so, j("oth.o"), j("td.o")])


def main():
    if sys.argv[1] == "--build-lib":
        build_library(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
        return
    src, dst, pats = sys.argv[1], sys.argv[2], sys.argv[3:]
    lines = open(src).read().split("\n")
    desc = descriptors(lines)
    for name, lo, hi in functions(lines):
        if any(p in name for p in pats):
            b, a = permute_function(lines, lo, hi, name, desc.get(name, {}))
            print("vgpr_banks: %s: bitop3 bank conflicts (hot loop, or body) %d -> %d" % (name, b, a))
    open(dst, "w").write("\n".join(lines))


if __name__ == "__main__":
    main()
