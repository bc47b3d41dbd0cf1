// bitboard.hpp — gfx950 device primitives for 8x8 Othello bitboards.
//
// Cost model (measured on MI355X, tools/diag/valu_rate*.cpp, DESIGN.md §Cost model):
// a kernel's throughput is the issue cost of its VALU instructions per env-step.
// Streamed alone, bitwise logic issues in ~2.2 cycles per wave64 and nearly
// everything else (64-bit shifts and adds, v_bfi/v_or3, v_bcnt, v_min,
// v_bfrev) in ~4-4.4; in these mixed loops a slow instruction costs ~6.5 at the
// margin and a fast one ~2.9 in a VOP3 encoding but ~3.7 in a VOP1/VOP2 one
// (tools/diag/valu_rate7.cpp).  Hence:
//   * 64-bit shifts and adds stay single v_lshl/v_lshrrev_b64 / v_lshl_add_u64;
//   * all 2- and 3-input logic (fill steps, masks, flip accumulation) is one
//     v_bitop3_b32 per 32-bit half (bitop3, bfi, andn, or3, and2, or2), and
//     the bit reversal and 32-bit shifts are written in their VOP3 forms;
//   * Kogge-Stone propagators are computed once per position and shared between
//     opposite directions (p2R = p2L >> S, p4R = p4L >> 3S);
//   * the chosen move's flips come from per-square ray tables in LDS and the
//     run sets of the analysis (flips_rays), not from more fills; without run
//     sets (the single step) from one carry along each ray (flips_carry).
//
// Square sq = x + 8*y (board.py:74-81); rays of board.py:9-17 as shifts:
//   +1 R (x+1), +8 D (y+1), +9 RD, +7 LD   and their opposites -1 L, -8 U, -9 LU, -7 RU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace oth {

typedef uint64_t u64;
typedef uint32_t u32;

constexpr u64 INNER_FILES = 0x7E7E7E7E7E7E7E7Eull;  // files b..g: a disc on a/h cannot be flanked along a row/diagonal

// any 3-input bitwise function as one v_bitop3_b32 per half.  TT is the
// function's value on (a, b, c) = (0xF0, 0xCC, 0xAA): 0xCA = a ? b : c,
// 0x80 = a & b & c, 0xFE = a | b | c, 0x30 = a & ~b, 0x20 = a & ~b & c,
// 0x04 = ~a & b & ~c.
template <int TT>
__device__ __forceinline__ u64 bitop3(u64 a, u64 b, u64 c) {
    // (the builtin returns int: take both halves as u32, no sign extension)
    const u32 hi = (u32)__builtin_amdgcn_bitop3_b32((u32)(a >> 32), (u32)(b >> 32), (u32)(c >> 32), TT);
    const u32 lo = (u32)__builtin_amdgcn_bitop3_b32((u32)a, (u32)b, (u32)c, TT);
    return ((u64)hi << 32) | lo;
}
// The three-input logic of these kernels goes through v_bitop3_b32 by hand:
// measured on the box (tools/diag/valu_rate5.cpp, 8 waves/SIMD) it issues in
// 2.4-2.5 cycles per wave-instruction where v_bfi_b32 and v_or3_b32 take 4.2,
// and hipcc emits bfi / or3 / bfi-with-0 for these forms on its own.
// bfi(m, a, b) = (m & a) | (~m & b).  Every Kogge-Stone step "gen |= pro &
// shifted" is written as bfi(pro, shifted, gen): the propagator never
// intersects the current fill (a propagator square at distance <= 2^k from the
// source would need an opponent disc at distance 0), so both forms agree.
__device__ __forceinline__ u64 bfi(u64 m, u64 a, u64 b) { return bitop3<0xCA>(m, a, b); }
__device__ __forceinline__ u64 andn(u64 a, u64 b) { return bitop3<0x30>(a, b, b); }
__device__ __forceinline__ u64 or3(u64 a, u64 b, u64 c) { return bitop3<0xFE>(a, b, c); }
// Two-input AND / OR as v_bitop3_b32 too (VOP3), not hipcc's v_and/v_or_b32_e32
// (VOP2).  Measured on the box (tools/diag/valu_rate7.cpp, 8 waves/SIMD): a
// fast instruction issued among slow VOP3 ones (64-bit shifts,
// v_lshl_add_u64, v_bcnt) costs ~2.9 cycles in a VOP3 encoding and ~3.6 in
// a VOP1/VOP2 one, though both stream at ~2.2 alone.
__device__ __forceinline__ u64 and2(u64 a, u64 b) { return bitop3<0xC0>(a, b, b); }
__device__ __forceinline__ u64 or2(u64 a, u64 b) { return bitop3<0xFC>(a, b, b); }
// 32-bit shifts by a constant in their VOP3 encoding (same reason)
template <int K, bool L>
__device__ __forceinline__ u32 sh32(u32 x) {
    u32 r;
    if (L) asm("v_lshlrev_b32_e64 %0, %2, %1" : "=v"(r) : "v"(x), "i"(K));
    else asm("v_lshrrev_b32_e64 %0, %2, %1" : "=v"(r) : "v"(x), "i"(K));
    return r;
}
// 64-bit shifts as single v_lshlrev_b64 / v_lshrrev_b64 (inline asm): with
// the 3-input logic taken apart into 32-bit halves, hipcc's combiner would
// otherwise split each shift into v_lshlrev_b32 + v_alignbit_b32, two
// instructions where one 64-bit shift issues as fast (valu_rate5.cpp).
template <int S, bool L>
__device__ __forceinline__ u64 sh(u64 x) {
    static_assert(S > 0 && S < 64, "shift amount");
    u64 r;
    if (L) asm("v_lshlrev_b64 %0, %2, %1" : "=v"(r) : "v"(x), "i"(S));
    else asm("v_lshrrev_b64 %0, %2, %1" : "=v"(r) : "v"(x), "i"(S));
    return r;
}

// Kogge-Stone propagators of one direction pair (+S / -S) for opponent set `pro`
struct PairProp {
    u64 pro, p2L, p4L, p2R, p4R;
};
template <int S>
__device__ __forceinline__ PairProp pair_prop(u64 pro) {
    PairProp q;
    q.pro = pro;
    q.p2L = and2(pro, sh<S, true>(pro));          // q, q-S in pro
    q.p4L = and2(q.p2L, sh<2 * S, true>(q.p2L));  // q .. q-3S in pro
    q.p2R = sh<S, false>(q.p2L);                 // q, q+S in pro
    q.p4R = sh<3 * S, false>(q.p4L);             // q .. q+3S in pro
    return q;
}

// one Kogge-Stone step gen |= pro & (gen shifted by K).  A shift by K >= 32
// moves one half into the other and leaves zeros behind, and a zero half of the
// shifted fill leaves that half of gen as it is: one 32-bit shift (none for
// K = 32) and one v_bitop3_b32, against a 64-bit shift and two bitop3.
template <int K, bool L>
__device__ __forceinline__ u64 ks_step(u64 gen, u64 pro) {
    if constexpr (K >= 32) {
        u32 lo = (u32)gen, hi = (u32)(gen >> 32);
        if (L) {
            const u32 s = K == 32 ? lo : sh32<(K == 32 ? 1 : K - 32), true>(lo);
            hi = (u32)__builtin_amdgcn_bitop3_b32((u32)(pro >> 32), s, hi, 0xCA);
        } else {
            const u32 s = K == 32 ? hi : sh32<(K == 32 ? 1 : K - 32), false>(hi);
            lo = (u32)__builtin_amdgcn_bitop3_b32((u32)pro, s, lo, 0xCA);
        }
        return ((u64)hi << 32) | lo;
    } else {
        return bfi(pro, sh<K, L>(gen), gen);
    }
}

// occluded fill of `gen` along +S (L) or -S through the pair's propagators:
// covers distances 0..7
template <int S, bool L>
__device__ __forceinline__ u64 ks(u64 gen, const PairProp& q) {
    gen = ks_step<S, L>(gen, q.pro);
    gen = ks_step<2 * S, L>(gen, L ? q.p2L : q.p2R);
    gen = ks_step<4 * S, L>(gen, L ? q.p4L : q.p4R);
    return gen;
}

// 64-bit adds as one v_lshl_add_u64 each (inline asm, for the same reason as
// sh: an add of a value assembled from halves is otherwise split in two)
__device__ __forceinline__ u64 lshl1_add(u64 x, u64 y) {  // (x << 1) + y
    u64 r;
    asm("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
__device__ __forceinline__ u64 add64(u64 x, u64 y) {
    u64 r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
__device__ __forceinline__ u64 dec64(u64 x) {  // x - 1
    u64 r;
    asm("v_lshl_add_u64 %0, %1, 0, -1" : "=v"(r) : "v"(x));
    return r;
}
// discs of `Oi` (inner opponent discs) in runs that start right east of a bit of
// `src`: the carry of Oi + (src << 1) ripples through each such run (one
// v_lshl_add_u64 + one v_bitop3_b32 per half); equal to the Kogge-Stone east
// fill from src through Oi, minus src.
__device__ __forceinline__ u64 east_run(u64 src, u64 Oi) { return andn(Oi, lshl1_add(src, Oi)); }

// 64-bit bit reversal (two v_bfrev_b32, halves swapped): square sq <-> 63 - sq,
// which turns the west ray into an east ray.
// v_bfrev_b32 in its VOP3 encoding (inline asm; hipcc emits the VOP1 one):
// a VOP1 slow instruction takes the VOP3 ones after it back to ~3.6 cycles
// (tools/diag/valu_rate7.cpp)
__device__ __forceinline__ u32 bfrev32(u32 x) {
    u32 r;
    asm("v_bfrev_b32_e64 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ u64 rev64(u64 x) { return ((u64)bfrev32((u32)x) << 32) | bfrev32((u32)(x >> 32)); }

// All propagators + attached runs of one position (mover P, opponent O).
// A[i]: opponent discs reachable from a P disc along direction i through
// opponent discs only (board.py:124-139's "hostile" runs, seen from P).
// Direction index i: 0:+1 1:-1 2:+8 3:-8 4:+9 5:-9 6:+7 7:-7
struct Position {
    u64 Oi, rOi;  // inner opponent discs, and bit-reversed
    u64 A[8];
    u64 reach;  // squares one step beyond an attached run (any content)
    u64 legal;  // Board.puttables as a mask (board.py:46-52) = reach & empty
};

// ORDER: the order the six Kogge-Stone fills are written in (digits = the
// direction pairs 7/8/9).  It only steers hipcc's register allocation: a
// v_bitop3_b32 whose three sources sit in one VGPR bank issues in 4.3 cycles
// instead of 2.5, and the bit pairs of 64-bit values make that likely; the
// order with the fewest such instructions in each kernel's hot loop was picked
// by tools/valu_mix.py (random rollout: 7-9-8, 11 -> 3 per ply).
constexpr int kFillOrder = 798;
template <int ORDER = kFillOrder>
__device__ __forceinline__ void analyse(u64 P, u64 O, Position& s) {
    const u64 Oi = and2(O, INNER_FILES);
    s.Oi = Oi;
    s.rOi = rev64(Oi);
    // the horizontal pair needs no propagators (carry tricks below)
    const PairProp v = pair_prop<8>(O), d9 = pair_prop<9>(Oi), d7 = pair_prop<7>(Oi);
    // east (+1): bits along the ray are contiguous, so one add propagates a
    // carry from each P disc through its adjacent run of inner opponent discs
    // and clears exactly those run bits: A = Oi & ~(Oi + (P << 1)).
    s.A[0] = east_run(P, Oi);
    // west (-1): the same on the bit-reversed board
    s.A[1] = rev64(east_run(rev64(P), s.rOi));
    // the Kogge-Stone fills from P stay inside P | O, so "minus P" is "and O"
    {
        constexpr int order[3] = {ORDER / 100, ORDER / 10 % 10, ORDER % 10};
#pragma unroll
        for (int k = 0; k < 3; k++) {
            if (order[k] == 8) {
                s.A[2] = and2(ks<8, true>(P, v), O);
                s.A[3] = and2(ks<8, false>(P, v), O);
            } else if (order[k] == 9) {
                s.A[4] = and2(ks<9, true>(P, d9), O);
                s.A[5] = and2(ks<9, false>(P, d9), O);
            } else {
                s.A[6] = and2(ks<7, true>(P, d7), O);
                s.A[7] = and2(ks<7, false>(P, d7), O);
            }
        }
    }
    // a legal square is one step beyond an attached run, and empty
    u64 m = or3(sh<1, true>(s.A[0]), sh<1, false>(s.A[1]), sh<8, true>(s.A[2]));
    m = or3(m, sh<8, false>(s.A[3]), sh<9, true>(s.A[4]));
    m = or3(m, sh<9, false>(s.A[5]), sh<7, true>(s.A[6]));
    m = or2(m, sh<7, false>(s.A[7]));
    s.reach = m;
    s.legal = bitop3<0x04>(P, m, O);  // ~P & m & ~O: one v_bitop3_b32 per half
}

// ---------------------------------------------------------------------------
// Flips from per-square ray tables (LDS).  For a ray R leaving the move square
// in increasing bit order, the flipped discs are the run-set squares A on R
// before the first square of R that is not in A:
//     x = R & ~A;   flips = R & A & (x - 1)
// (x != 0 whenever R & A != 0: an attached run ends in a P disc on the same ray).
// Rays that leave in decreasing bit order use the same identity on the
// bit-reversed board.  Table rows: 0..2 = rays +8, +9, +7 (normal order),
// 3..5 = rays -8, -9, -7 stored bit-reversed; 64 squares each (3 KiB).
constexpr int kRayRows = 6;
// the LDS table adds two rows per square: 6 = the square's bit, 7 = its bit
// on the reversed board (1 << (63 - sq)); read with the rays, they replace two
// variable 64-bit shifts of the VALU-bound loop by LDS reads
constexpr int kTabRows = kRayRows + 2;
__host__ __device__ inline u64 ray_from(int sq, int dx, int dy) {
    u64 r = 0;
    int x = sq & 7, y = sq >> 3;
    for (;;) {
        x += dx;
        y += dy;
        if (x < 0 || x > 7 || y < 0 || y > 7) break;
        r |= 1ull << (x + 8 * y);
    }
    return r;
}
__device__ __forceinline__ void ray_table_init(u64* tab) {
    for (int e = threadIdx.x; e < kTabRows * 64; e += blockDim.x) {
        const int row = e >> 6, sq = e & 63;
        const int dx[6] = {0, 1, -1, 0, -1, 1}, dy[6] = {1, 1, 1, -1, -1, -1};
        if (row >= kRayRows) {
            tab[e] = 1ull << (row == kRayRows ? sq : 63 - sq);
            continue;
        }
        const u64 r = ray_from(sq, dx[row], dy[row]);
        tab[e] = row < 3 ? r : rev64(r);
    }
}
// the move's bit from the table (row kRayRows)
__device__ __forceinline__ u64 square_bit(u32 sq, const u64* tab) { return tab[kRayRows * 64 + sq]; }
__device__ __forceinline__ u64 and3(u64 a, u64 b, u64 c) { return bitop3<0x80>(a, b, c); }
// For a ray R leaving the move in increasing bit order and the run set A of
// the opposite direction, the flipped discs are the squares of R before R's
// first square that is not in A: with x = R & ~A, R & A & (x - 1).  (x - 1)
// sets the bits below x's lowest bit but keeps x's higher bits, so the "& A"
// is needed.
__device__ __forceinline__ u64 run_prefix(u64 R, u64 A) {
    const u64 x = andn(R, A);
    return and3(R, A, dec64(x));
}

// The run sets flips_rays reads, in the orientation it reads them: the runs
// leaving a move in increasing bit order lie in A[1], A[3], A[5], A[7] (the
// opposite directions' runs, as analyse gives them), those leaving in
// decreasing order in A[0], A[2], A[4], A[6], kept bit-reversed.  The 1-ply
// policies build this once per parent and share it among its children.
struct RunSets {
    u64 A1, A3, A5, A7, rA0, rA2, rA4, rA6;
};
__device__ __forceinline__ RunSets run_sets(const Position& s) {
    return RunSets{s.A[1], s.A[3], s.A[5], s.A[7], rev64(s.A[0]), rev64(s.A[2]), rev64(s.A[4]), rev64(s.A[6])};
}

// The flips of the move at square sq (bit mv) in two parts, both including
// the move's own bit: f in the normal orientation (east and the rays leaving
// in increasing bit order) and fr for the rays leaving in decreasing order,
// computed on the bit-reversed board and reversed back once.  Horizontal: the
// run of A[1] that starts right east of the move is exactly its east flips
// (an A[1] run is attached to a P disc on its far side and bounded by the
// empty move square on this side; A runs lie on the inner files, so the carry
// never leaves the row): one add, as east_run, and the move's bit ORed in by
// the same v_bitop3_b32.  West the same on the reversed board with A[0].  The
// other six by the ray tables (run_prefix).  place() applies both parts: the
// move's bit is never an opponent disc, so carrying it in the flips costs
// nothing and saves the apply's separate OR.
struct Flips {
    u64 f, fr;
};
// col = tab + sq: the move's column of the table (rows 64 entries apart)
__device__ __forceinline__ Flips flips_col(u64 mv, const RunSets& r, const u64* col) {
    const u64 rmv = col[(kRayRows + 1) * 64];
    u64 f = bitop3<0xBA>(r.A1, lshl1_add(mv, r.A1), mv);     // (A1 & ~(A1 + (mv << 1))) | mv
    u64 fr = bitop3<0xBA>(r.rA0, lshl1_add(rmv, r.rA0), rmv);  // west, in reversed space
    f = or3(f, run_prefix(col[0 * 64], r.A3), run_prefix(col[1 * 64], r.A5));
    f = or2(f, run_prefix(col[2 * 64], r.A7));
    fr = or3(fr, run_prefix(col[3 * 64], r.rA2), run_prefix(col[4 * 64], r.rA4));
    fr = or2(fr, run_prefix(col[5 * 64], r.rA6));
    return Flips{f, rev64(fr)};
}
__device__ __forceinline__ Flips flips_rays(u32 sq, const RunSets& r, const u64* tab) {
    return flips_col(tab[kRayRows * 64 + sq], r, tab + sq);
}
// the move: mover X |= flips | mv, opponent Y &= ~flips
__device__ __forceinline__ void place(u64& X, u64& Y, const Flips& fl) {
    X = or3(X, fl.f, fl.fr);
    Y = bitop3<0x10>(Y, fl.f, fl.fr);  // Y & ~f & ~fr
}
// the column of the square whose byte offset kth_bit_off returned
__device__ __forceinline__ const u64* ray_col(const u64* tab, u32 off) {
    return reinterpret_cast<const u64*>(reinterpret_cast<const char*>(tab) + off);
}

// ---------------------------------------------------------------------------
// Flips of one move without run sets (the single-step kernel, where the mover's
// analysis is not otherwise needed).  Along a ray R leaving the move in
// increasing bit order, the carry of X + mv, X = (O | ~R), starts at the move's
// own bit (set in X: the move is not on its ray), ripples through the non-ray
// bits up to R's first square, on through the opponent discs at the start of
// the ray (and the non-ray bits between them), and stops on the first ray
// square that is not an opponent disc, which it sets.  The opponent squares it
// cleared are the run; they flip iff the stop square holds a P disc.  A run
// that reaches the edge carries out of the ray: no stop square, no flips.
// Round 5: the carry starts at mv, not at the ray's first square (six variable
// 64-bit shifts fewer), and the diagonal rays are the shifted line patterns
// unmasked, with O taken on the inner files only (Oi): an opponent disc on an
// edge file can never be flanked along a diagonal, so the stop is at the
// ray's edge square at the latest, before any square the pattern wraps to; a
// move on the edge file, whose exact ray is empty, stops at once on a wrapped
// square with an empty run.  That drops the two file masks and their
// reversals (2 shifts, 2 adds, 4 v_bfrev, 8 v_bitop3).
// The test is one 64-bit compare (v_cmp_ne_u64) and the select two
// v_cndmask: hipcc ORs the two halves of the and3 and compares 32 bits.
__device__ __forceinline__ u64 sel_nz(u64 t, u64 x) {  // t != 0 ? x : 0
    u32 lo, hi;
    u64 m;
    asm("v_cmp_ne_u64_e64 %2, 0, %3\n\t"
        "s_nop 1\n\t"
        "v_cndmask_b32_e64 %0, 0, %4, %2\n\t"
        "v_cndmask_b32_e64 %1, 0, %5, %2"
        : "=&v"(lo), "=&v"(hi), "=&s"(m)  // early-clobber: lo is written before x's high half is read
        : "v"(t), "v"((u32)x), "v"((u32)(x >> 32)));
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 ray_flips(u64 mv, u64 R, u64 P, u64 O) {
    const u64 sum = add64(bfi(R, O, ~0ull), mv);  // (O | ~R) + mv
    const u64 run = bitop3<0x20>(R, sum, O);      // R & ~sum & O
    return sel_nz(and3(sum, R, P), run);          // stop square is P
}

// The six rays of one square in registers: rows 0..2 the increasing rays +8,
// +9, +7, rows 3..5 the decreasing ones in the bit-reversed layout (square
// 63 - sq).  The diagonals are the shifted line patterns, unmasked (see
// ray_flips: their carries run over the inner-file opponent discs).  Six
// v_lshlrev_b64; the single-step kernel uses this instead of an LDS table,
// whose per-block copy and barrier cost more (tools/diag/launch_floor.py,
// step_ab.py), or a constant table in global memory: six more vector loads
// per board cost the HBM-bound step 159 -> 182 us per 16M boards (round 4).
__device__ __forceinline__ void rays_of(u32 sq, u64 (&R)[kRayRows]) {
    const u32 rsq = sq ^ 63u;
    R[0] = 0x0101010101010100ull << sq;   // +8
    R[1] = 0x8040201008040200ull << sq;   // +9 (wraps past file h: see ray_flips)
    R[2] = 0x0002040810204080ull << sq;   // +7 (wraps past file a)
    R[3] = 0x0101010101010100ull << rsq;  // -8, reversed
    R[4] = 0x8040201008040200ull << rsq;  // -9, reversed
    R[5] = 0x0002040810204080ull << rsq;  // -7, reversed
}

// flips of the move on empty square sq (Board.put's count is their popcount,
// board.py:161-174); 0 when nothing is flanked.  Exact for any disjoint own /
// opponent pair (put_s_any's Empty side included).  Horizontal runs by the
// carry on the inner files, the six others by ray_flips (the diagonals over
// the inner files, the verticals over all); rays leaving in decreasing bit
// order on the bit-reversed board.
__device__ __forceinline__ u64 flips_carry(u32 sq, u64 P, u64 O) {
    u64 R[kRayRows];
    rays_of(sq, R);
    const u64 mv = 1ull << sq, rmv = 1ull << (63u - sq);
    const u64 rP = rev64(P), rO = rev64(O);
    const u64 Oi = and2(O, INNER_FILES), rOi = and2(rO, INNER_FILES);
    const u64 se = lshl1_add(mv, Oi), sw = lshl1_add(rmv, rOi);
    u64 f = sel_nz(and2(se, P), andn(Oi, se));
    u64 fr = sel_nz(and2(sw, rP), andn(rOi, sw));
    f = or3(f, ray_flips(mv, R[0], P, O), ray_flips(mv, R[1], P, Oi));
    f = or2(f, ray_flips(mv, R[2], P, Oi));
    fr = or3(fr, ray_flips(rmv, R[3], rP, rO), ray_flips(rmv, R[4], rP, rOi));
    fr = or2(fr, ray_flips(rmv, R[5], rP, rOi));
    return or2(f, rev64(fr));
}

// legal moves only (no run sets kept) — for child positions / next-state masks
template <int ORDER = kFillOrder>
__device__ __forceinline__ u64 moves(u64 P, u64 O) {
    Position s;
    analyse<ORDER>(P, O, s);
    return s.legal;
}

// Board.puttables(Empty) (board.py:46-52 with piece = Empty, hostile(Empty) =
// Black, 155-159): empty squares from which a run of >= 1 black disc ends on an
// empty square -- the mobility counts() reports for a side string other than
// 'O'/'X' (turn_from_string -> Empty, board.py:245-251).
__device__ __forceinline__ u64 moves_empty_side(u64 black, u64 white) {
    const u64 E = ~(black | white);
    Position s;
    analyse(E, black, s);
    return s.reach & E;
}

// k-th set bit via two popcount bisection levels (32, 16, 8) and a 256x8 byte
// table in LDS: tab[b * 8 + k] = index of the k-th set bit of byte b.
__device__ __forceinline__ void kth_table_init(uint8_t* tab) {
    for (int b = threadIdx.x; b < 256; b += blockDim.x) {
        int k = 0;
        for (int i = 0; i < 8; i++)
            if (b >> i & 1) tab[b * 8 + k++] = (uint8_t)i;
        for (; k < 8; k++) tab[b * 8 + k] = 0;
    }
}
// (a + b) << 3 as one v_add_lshl_u32 (hipcc otherwise distributes the shift
// over the terms of a, one v_lshlrev_b32 each)
__device__ __forceinline__ u32 add_lshl3(u32 a, u32 b) {
    u32 r;
    asm("v_add_lshl_u32 %0, %1, %2, 3" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// c_lo = __popc((u32)x), which the caller has from counting x (popcount_lo).
// Returns 8 x the square: the byte offset of the square's entries in the LDS
// ray table.  Each level keeps k as k or k - c by the subtraction's borrow
// (kth_level; formerly min(k, k - c)), the byte is one v_bfe_u32 at the last
// level's offset, and the three level offsets are disjoint bits (32 | 16 | 8):
// one v_or3 and one v_add_lshl with the table entry give the offset
// (31 -> 24 VALU per pick with the address arithmetic).
// One bisection level in VOP3 with the borrow as the select: b = (k < c) from
// v_sub_co_u32's borrow, k = b ? k : k - c and off = b ? 0 : S by two
// v_cndmask_b32_e64, where min(k, k - c) cost a v_min_u32 (a slow
// instruction, ~6.5 cycles at the margin in this loop; a v_cndmask_b32_e64
// among v_bitop3_b32 costs ~2.7: tools/diag/valu_rate7.cpp).  The s_nop gives
// the two wait states a VALU-written SGPR needs before a VALU reads it (hipcc
// puts one instruction and an s_nop 0 there).  W: w = b ? w_lo : w_hi (the
// 32-bit level's word select), else unused.
template <int S, bool W>
__device__ __forceinline__ void kth_level(u32& k, u32 c, u32& off, u32& w, u32 w_hi) {
    u32 d, k2, o, w2;
    u64 b;
    if (W)
        asm("v_sub_co_u32_e64 %0, %4, %5, %6\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e64 %1, %0, %5, %4\n\t"
            "v_cndmask_b32_e64 %2, %7, 0, %4\n\t"
            "v_cndmask_b32_e64 %3, %9, %8, %4"
            : "=&v"(d), "=&v"(k2), "=&v"(o), "=v"(w2), "=&s"(b)
            : "v"(k), "v"(c), "i"(S), "v"(w), "v"(w_hi));
    else
        asm("v_sub_co_u32_e64 %0, %3, %4, %5\n\t"
            "s_nop 1\n\t"
            "v_cndmask_b32_e64 %1, %0, %4, %3\n\t"
            "v_cndmask_b32_e64 %2, %6, 0, %3"
            : "=&v"(d), "=&v"(k2), "=v"(o), "=&s"(b)
            : "v"(k), "v"(c), "i"(S));
    k = k2;
    off = o;
    if (W) w = w2;
}
__device__ __forceinline__ u32 kth_bit_off(u64 x, u32 k, u32 c_lo, const uint8_t* tab) {
    u32 w = (u32)x, b32, s16, s8;
    kth_level<32, true>(k, c_lo, b32, w, (u32)(x >> 32));
    kth_level<16, false>(k, __popc(w & 0xFFFFu), s16, w, 0u);
    w >>= s16;
    kth_level<8, false>(k, __popc(w & 0xFFu), s8, w, 0u);
    const u32 byte = __builtin_amdgcn_ubfe(w, s8, 8);
    // the disjoint level offsets ORed by one v_bitop3_b32 (hipcc's v_or3_b32 is slow)
    const u32 lvl = (u32)__builtin_amdgcn_bitop3_b32(b32, s16, s8, 0xFE);
    return add_lshl3(lvl, tab[byte * 8u + k]);
}
__device__ __forceinline__ u32 kth_bit_tab(u64 x, u32 k, u32 c_lo, const uint8_t* tab) {
    return kth_bit_off(x, k, c_lo, tab) >> 3;
}

// index of the k-th set bit (LSB-first, 0-based) of x; requires k < popcount(x).
__device__ __forceinline__ u32 kth_bit(u64 x, u32 k) {
    u32 lo = (u32)x, hi = (u32)(x >> 32);
    u32 c = __popc(lo);
    bool up = k >= c;
    u32 w = up ? hi : lo;
    k = up ? k - c : k;
    u32 pos = up ? 32u : 0u;
#pragma unroll
    for (int half = 16; half >= 1; half >>= 1) {
        const u32 mask = (1u << half) - 1u;
        c = __popc(w & mask);
        up = k >= c;
        w = up ? (w >> half) : w;
        k = up ? k - c : k;
        pos += up ? (u32)half : 0u;
    }
    return pos;
}

}  // namespace oth
