// othello.hip — MI355X (gfx950) kernels + C-ABI for the batched Othello env.
//
// Replaces the step path of ysnrkdm/subproc board.py:
//   puttables / n_puttable_for  (board.py:46-55)   -> moves(): Kogge-Stone fills + carry rays
//   put / put_s                 (board.py:161-209) -> step: flips_carry; rollouts: flips_rays
//                                                     (LDS ray table + run-set prefix)
//   is_game_over                (board.py:57-58)   -> two-pass rule in the rollout loop
//   n_black / n_white + result  (board.py:37-41, game_runner.py:194-199)
//   play loop                   (game_runner.py:165-201) -> rollout_kernel
// and the §8f rows beside it: replay + book text (game_recorder.py), counts()
// features, the learner's linear eval, eval-table self-play / matches, and the
// TD state-map update (progress_position_moves_learn.py:37-62).
//
// Design: one game per lane, state in VGPRs as two uint64 bitboards
// (mover P, opponent O); pure integer/bitwise VALU work, no MFMA.  The cost of
// a rollout is its VALU instruction count per env-step (bitboard.hpp), so the
// rollout kernel keeps per-iteration control flow minimal: a wave dequeues 64
// game ids (one per lane) from a per-launch counter, plays them out with
// __ballot-driven lane masking, then dequeues again.  LDS holds the k-th-bit
// byte table, the ray table, the per-workgroup win/score histogram (one global
// atomic per non-zero bin per workgroup at exit) and, for the 1-ply policies,
// the per-wave cooperative child list (coop_choose).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <atomic>
#include <mutex>

#include "../../include/othello.h"
#include "bitboard.hpp"
#include "td_skey.hpp"

#define OTH_VERSION "subproc_amd 0.1.0 gfx950"

namespace {

using namespace oth;

constexpr u64 OPEN_BLACK = 0x0000000810000000ull;  // e4, d5  (board.py:25)
constexpr u64 OPEN_WHITE = 0x0000001008000000ull;  // d4, e5  (board.py:24)
constexpr int kBlock = 256;

// ---------------------------------------------------------------------------
// RNG spec (twins: oracle/othello_oracle.c, tests/golden/gen_golden.py)
// ---------------------------------------------------------------------------
constexpr u64 GOLDEN64 = 0x9E3779B97F4A7C15ull;
__host__ __device__ __forceinline__ u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ u64 game_key(u64 S, u64 g) { return mix64(S + g * GOLDEN64); }
// per-game draw stream: 32-bit LCG, state0 = lo32(key), increment = hi32(key) | 1;
// a uniform pick in [0, n) is umulhi(draw, n)
constexpr u32 LCG_MUL = 0x915F77F5u;
struct GameRng {
    u32 state, inc;
    __device__ __forceinline__ void init(u64 key) {
        state = (u32)key;
        inc = (u32)(key >> 32) | 1u;
    }
    __device__ __forceinline__ u32 pick(u32 n) {
        state = state * LCG_MUL + inc;
        return __umulhi(state, n);
    }
};
// the random rule's move: the k-th legal square, k uniform in [0, popcount)
// (the low word's count is shared by the total and the k-th-bit search)
__device__ __forceinline__ u32 pick_legal(u64 legal, GameRng& rng, const uint8_t* kth_tab) {
    const u32 c_lo = __popc((u32)legal);
    return kth_bit_tab(legal, rng.pick(c_lo + __popc((u32)(legal >> 32))), c_lo, kth_tab);
}


// counts() region masks a..h (parameter_progress_position_moves_learn.py:9-16)
__constant__ u64 kRegionMasks[8] = {0x8100000000000081ull, 0x4281000000008142ull, 0x0042000000004200ull,
                                    0x2400810000810024ull, 0x1800008181000018ull, 0x003C424242423C00ull,
                                    0x0000240000240000ull, 0x0000183C3C180000ull};

// Linear eval (§8f row 2).  Weights: int8 [4][9] (include/othello.h), held as
// int32 rows padded to 12 in LDS / registers.  The shard of a disc count d is
// (d - 1) >> 4 for d in 1..64 (shards 0..16, 17..32, 33..48, 49..64 of
// progress_position_moves_learn.py:112-113).
constexpr int kEvalRow = 12;
constexpr int kEvalTable = OTH_EVAL_PHASES * kEvalRow;
struct EvalWeights {
    int8_t w[OTH_EVAL_WEIGHTS];
};
__device__ __forceinline__ u32 eval_shard(u32 discs) { return discs ? (min(discs, 64u) - 1u) >> 4 : 0u; }
__device__ __forceinline__ void eval_weights_to_lds(const EvalWeights& ew, int* w_s) {
    for (int e = threadIdx.x; e < OTH_EVAL_PHASES * kEvalRow; e += blockDim.x) {
        const int r = e / kEvalRow, c = e % kEvalRow;
        w_s[e] = c < OTH_EVAL_FEATURES ? (int)ew.w[r * OTH_EVAL_FEATURES + c] : 0;
    }
}
// sum_j w[j] * counts()[1+j] for the side owning `mine`, with mobility `mob`
// The products by 24-bit multiplies (v_mul_i32_i24, full rate) where a plain
// int multiply is v_mul_lo_u32, a multi-pass instruction: the weights are
// int8 and the counts <= 64, so every product and partial sum is exact in
// 24 bits.
__device__ __forceinline__ int eval_mul(int w, int c) { return __mul24(w, c); }
__device__ __forceinline__ int eval_linear(const int* w, u64 mine, u64 mob) {
    int v = eval_mul(w[0], (int)__popcll(mob));
#pragma unroll
    for (int k = 0; k < 8; k++) v += eval_mul(w[1 + k], (int)__popcll(and2(mine, kRegionMasks[k])));
    return v;
}

// ---------------------------------------------------------------------------
// 1-ply policies (greedy: minimise the opponent's mobility on the child; eval:
// maximise the mover's linear eval of the child; ties -> lowest square, the
// first in puttables order).  A child's score is a key whose minimum is the
// choice: (score << 6) | square.  The parent then plays the chosen square
// itself (one flip computation): handing the best child's boards over through
// LDS instead cost more than it saved (round 4 A/B on one box, 1,048,576 games:
// greedy 2.245 / 2.226 ms with the hand-over, pipelined or not, against
// 2.183 ms without; eval 4.123 / 4.364 against 3.960 ms).
//
// the eval weight row of a parent's children: every child has popcount(P|O) + 1
// discs, so one row serves all of them (its address found once per parent;
// the weights themselves are read per child: held in registers they pushed
// the eval kernel past its 128 VGPRs)
template <int POLICY>
__device__ __forceinline__ const int* child_row(u64 P, u64 O, const int* w_tab) {
    if (POLICY != OTH_POLICY_EVAL) return w_tab;
    return w_tab + kEvalRow * eval_shard((u32)__popcll(P | O) + 1u);
}
template <int POLICY>
__device__ __forceinline__ u32 child_key(u64 P, u64 O, const RunSets& s, u32 sq, const u64* rays, const int* row) {
    place(P, O, flips_rays(sq, s, rays));
    if (POLICY == OTH_POLICY_GREEDY) return ((u32)__popcll(moves(O, P)) << 6) | sq;
    int w[OTH_EVAL_FEATURES];
#pragma unroll
    for (int j = 0; j < OTH_EVAL_FEATURES; j++) w[j] = row[j];
    // |v| < 2^14; fill order 7-9-8 (bitboard.hpp analyse): 9 same-bank v_bitop3_b32 in
    // this child loop against 13 at 8-7-9, +2-4% eval env-steps/s (tools/diag/r03_evalorder.sh)
    const int v = eval_linear(w, P, moves<798>(P, O));
    return ((u32)((1 << 20) - v) << 6) | sq;
}

// one lane alone over its own children (w_tab: the mover's eval table)
template <int POLICY>
__device__ __forceinline__ u32 lane_choose(const Position& pos, u64 P, u64 O, const u64* rays, const int* w_tab) {
    u32 best = 0xFFFFFFFFu;
    u64 legal = pos.legal;
    const RunSets s = run_sets(pos);
    const int* row = child_row<POLICY>(P, O, w_tab);
    while (legal) {
        const u32 sq = (u32)__builtin_ctzll(legal);  // legal != 0
        legal &= legal - 1;
        best = min(best, child_key<POLICY>(P, O, s, sq, rays, row));
    }
    return best & 63u;
}

// Wave-cooperative choice.  A lane's own child loop makes the wave pay for its
// busiest lane every ply (measured on greedy games: 662 child evaluations per
// 64-game batch where 303 would do, 46% lane efficiency).  Instead the wave's
// T children, numbered parent by parent in lane order (an exclusive scan of
// the lanes' move counts), are cut into 64 consecutive chunks of
// R = ceil(T / 64): lane i evaluates children R*i .. R*i + R - 1 in R rounds
// (finished games included).  A lane finds its chunk's first parent by a
// binary search of the scan and skips that parent's first children by the
// k-th-bit pick; from there it walks the parents' legal masks lowest square
// first, moving to the next parent with moves when one runs out.  A chunk
// spans one or two parents mostly, so the lane holds its current parent's
// record (and eval weight row) in registers and reads the next one from LDS
// only when it moves on.  Every choosing lane publishes its position (P, O,
// run sets) and legal mask to the wave's LDS area; each child's key is folded
// into its parent's slot with an LDS atomicMin (the order of evaluation does
// not matter).  (Round 3 listed each lane's surplus children in an overflow
// list, one entry per loop iteration of the busiest lane, ~13 VALU each; the
// chunks need no list.)  cap == 0 (OTH_COOP_CAP=0, tests) takes lane_choose
// for every choosing lane instead.
// (Round 5 A/B, not shipped: a mover with exactly one legal move playing it
// without scoring its child cut greedy VALU by 0.9% but ran 1.3% (greedy) /
// 5% (eval) slower per launch; tools/diag/r05_variants.patch.)
struct CoopWave {
    u64 rec[64][10];  // parent lane: P, O, its RunSets (8 words; A1's bit 0, a1, carries the eval table)
    u64 legal[64];    // parent lane's legal mask (0: not choosing)
    u32 best[64];
};
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
static_assert(sizeof(RunSets) == 8 * sizeof(u64), "parent record: P, O, RunSets");
__device__ __forceinline__ void load_parent(const u64* r, u64& P, u64& O, RunSets& s) {
    P = r[0];
    O = r[1];
    s = *reinterpret_cast<const RunSets*>(r + 2);
}
// inclusive scan over the wave's 64 lanes (DPP row shifts, then the row
// broadcasts of lanes 15 and 31)
__device__ __forceinline__ u32 wave_incl_scan(u32 x) {
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
// w_s: the two eval tables (kEvalTable ints each); tbl (0 / 1) is the mover's
// (Black's / White's, or in a GameRunner match player A's / B's).  Returns
// the chosen square of a choosing lane (64 otherwise).
// The table bit rides in bit 0 (square a1) of the record's A1, the west runs
// of inner opponent discs, which never holds a1; a stray bit 0 in A1 does not
// change flips_col's east carry either (bit 0 of mv << 1 is 0: no carry).
template <int POLICY>
__device__ u32 coop_choose(bool need, u64 P, u64 O, u32 tbl, const Position& pos, CoopWave& cw, const u64* rays,
                           const int* w_s, const uint8_t* kth_tab, u32 lane, u32 cap) {
    auto publish = [&] {
        u64* r = cw.rec[lane];
        r[0] = P;
        r[1] = O;
        RunSets rs = run_sets(pos);  // reversed once per parent, not per child
        if (POLICY == OTH_POLICY_EVAL) rs.A1 |= (u64)(tbl & 1u);
        *reinterpret_cast<RunSets*>(r + 2) = rs;
    };
    // greedy (round 6): the record first, on either path, since the caller
    // plays the chosen move from it
    constexpr bool kFirst = POLICY == OTH_POLICY_GREEDY;
    if (kFirst && need) publish();
    if (cap == 0) return need ? lane_choose<POLICY>(pos, P, O, rays, w_s + (tbl ? kEvalTable : 0)) : 64u;
    const u64 legal = need ? pos.legal : 0ull;
    const u32 cnt = (u32)__popcll(legal);
    const u32 incl = wave_incl_scan(cnt);
    const u32 T = (u32)__builtin_amdgcn_readlane((int)incl, 63);
    const u32 R = (T + 63u) >> 6;
    cw.legal[lane] = legal;
    if (need) {
        if (!kFirst) publish();
        cw.best[lane] = 0xFFFFFFFFu;
    }
    // this lane's chunk of the children: [t0, t0 + cnt_mine).  Its first
    // parent, the last lane whose first child is <= t0, by a binary search of
    // the exclusive scan, read from the lanes' registers by permutes (every
    // lane active); the parents with moves as one wave-uniform mask
    const u32 t0 = R * lane, cnt_mine = t0 < T ? min(R, T - t0) : 0u;
    const u32 excl = incl - cnt;
    const u64 with_moves = __ballot(cnt != 0);
    u32 p = 0;
#pragma unroll
    for (u32 step = 32; step >= 1; step >>= 1)
        if ((u32)__shfl((int)excl, (int)(p + step)) <= t0) p += step;
    const u32 k0 = t0 - (u32)__shfl((int)excl, (int)p);
    wave_sync();
    // the current parent: its remaining squares m, its record and weight row,
    // held across its children.  Round 4's eval kernel reread the record from
    // LDS per child (held, it spills a few per-batch values at its 128
    // VGPRs): that reread on every child's dependency chain is what made
    // eval on chunks 3.5% slower than round 3's surplus list, whose lanes
    // mostly evaluated their own children (PMC: same VALU per child within
    // 2%, round 5, profiles/r05_notes.md); held, eval runs at round 3's speed
    // (3.810 against 3.817 ms per 1M-game launch, 3.945 rereading)
    u64 m = 0, Pp = 0, Op = 0;
    RunSets ps = {};
    const int* row = w_s;
    auto enter = [&](u32 q) {
        load_parent(cw.rec[q], Pp, Op, ps);
        row = child_row<POLICY>(Pp, Op, w_s + ((ps.A1 & 1ull) ? kEvalTable : 0));
    };
    if (cnt_mine) {
        m = cw.legal[p];
        enter(p);
        if (k0) m &= ~0ull << kth_bit_tab(m, k0, (u32)__popc((u32)m), kth_tab);  // skip the chunk's predecessors
    }
    for (u32 r = 0; r < cnt_mine; r++) {
        if (m == 0) {  // the next parent with moves (one exists, above p < 63: t0 + r < T)
            p = (u32)__ffsll((unsigned long long)(with_moves & (~0ull << (p + 1)))) - 1u;
            m = cw.legal[p];
            enter(p);
        }
        const u32 sq = (u32)__builtin_ctzll(m);  // m != 0 here: no zero case (__ffsll's select)
        m &= m - 1;
        atomicMin(&cw.best[p], child_key<POLICY>(Pp, Op, ps, sq, rays, row));
    }
    wave_sync();
    return need ? cw.best[lane] & 63u : 64u;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ u64 moves_of(u64 P, u64 O) { return moves(P, O); }

// ---------------------------------------------------------------------------
// elementwise kernels
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void reset_kernel(u64* __restrict__ boards, uint8_t* __restrict__ turn,
                                                       uint8_t* __restrict__ nturn, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    reinterpret_cast<ulonglong2*>(boards)[i] = make_ulonglong2(OPEN_BLACK, OPEN_WHITE);
    if (turn) turn[i] = OTH_BLACK;
    if (nturn) nturn[i] = 0;
}

// ---------------------------------------------------------------------------
// Any side to move.  board.py's turn is Black or White in play, but Empty is
// reachable through deserialize with a side string other than 'O'/'X'
// (turn_from_string, board.py:245-251), and put/puttables take any piece.
// For a piece p the scan of hands_for_direc (board.py:124-139) collects
// squares holding hostile(p) (White for Black, else Black: 155-159) up to a
// square holding p.  So:
//   p = Black / White : the usual rule;
//   p = Empty (0)     : own squares = the empty squares, opponent = Black; a
//                       run of Black discs ended by an empty square is
//                       "flipped" to Empty, the origin stays Empty;
//   p >= 3            : no square holds p, nothing is ever flanked.
// put_s then toggles the turn to White if it was Black, else to Black (205-208).
// ---------------------------------------------------------------------------
__device__ __forceinline__ u64 legal_any(u64 bl, u64 wh, u32 t) {
    if (t == OTH_BLACK) return moves(bl, wh);
    if (t == OTH_WHITE) return moves(wh, bl);
    if (t == 0) return moves_empty_side(bl, wh);
    return 0ull;
}

struct StepOut {
    u64 bl, wh, flips;
    u32 t;
    int ret;
};
// put_s (board.py:192-209) on an integer move code for any side code t
__device__ __forceinline__ StepOut put_s_any(u64 bl, u64 wh, u32 t, u32 c) {
    const u64 occ = bl | wh;
    const bool black = t == OTH_BLACK, white = t == OTH_WHITE;
    const u64 own = black ? bl : (white ? wh : (t == 0 ? ~occ : 0ull));
    const u64 opp = black ? wh : bl;
    StepOut o{bl, wh, 0ull, t, -1};
    if (c == OTH_PASS) {
        o.ret = 0;
    } else if (c < 64 && !(occ >> c & 1ull)) {
        const u64 f = flips_carry(c, own, opp);  // exact for any own/opp pair (bitboard.hpp)
        if (f) {
            const u64 mv = 1ull << c;
            o.ret = __popcll(f);
            o.flips = f;
            if (black) {
                o.bl = or3(bl, f, mv);
                o.wh = andn(wh, f);
            } else if (white) {
                o.wh = or3(wh, f, mv);
                o.bl = andn(bl, f);
            } else {
                o.bl = andn(bl, f);  // set_hands / set with piece Empty
            }
        }
    }
    if (o.ret >= 0) o.t = black ? OTH_WHITE : OTH_BLACK;
    return o;
}

__global__ __launch_bounds__(kBlock) void legal_kernel(const u64* __restrict__ boards,
                                                       const uint8_t* __restrict__ turn, u64* __restrict__ legal,
                                                       int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(boards)[i];
    legal[i] = legal_any(b.x, b.y, turn[i]);
}

// one board of the step (board.py:192-209 semantics, see include/othello.h)
__device__ __forceinline__ void step_board(int64_t i, ulonglong2 b, u32 t, u32 mvc, u64* boards_out, uint8_t* turn_out,
                                           u64* __restrict__ flips_out,
                                           u64* __restrict__ legal_next, int8_t* __restrict__ ret_out,
                                           uint8_t* __restrict__ nturn) {
    u64 nb, nw, f = 0, lg = 0;
    u32 t_out;
    int r = -1;
    if (t == OTH_BLACK || t == OTH_WHITE) {
        const bool black = t == OTH_BLACK;
        u64 P = black ? b.x : b.y;
        u64 O = black ? b.y : b.x;
        if (mvc == OTH_PASS) {
            r = 0;
        } else if (mvc < 64) {
            const u64 mv = 1ull << mvc;
            if (!((P | O) & mv)) {
                f = flips_carry(mvc, P, O);
                if (f) {
                    r = __popcll(f);
                    P = or3(P, f, mv);
                    O = andn(O, f);
                }
            }
        }
        const bool moved = r >= 0;
        t_out = moved ? (t ^ 3u) : t;
        // one analysis of whichever side moves next (select the operands, not
        // the results): O if the turn toggled
        if (legal_next) {
            const u64 nP = moved ? O : P, nO = moved ? P : O;
            lg = moves(nP, nO);
        }
        nb = black ? P : O;
        nw = black ? O : P;
    } else {
        // side to move Empty (or no colour at all): rare, off the fast path
        const StepOut o = put_s_any(b.x, b.y, t, mvc);
        nb = o.bl;
        nw = o.wh;
        f = o.flips;
        r = o.ret;
        t_out = o.t;
        if (legal_next) lg = legal_any(nb, nw, t_out);
    }
    // streaming outputs: non-temporal stores (tools/diag/step_ab.py at 16M
    // boards: 157 against 161 us with ordinary stores)
    if (legal_next) __builtin_nontemporal_store(lg, legal_next + i);
    if (boards_out) {
        __builtin_nontemporal_store(nb, boards_out + 2 * i);
        __builtin_nontemporal_store(nw, boards_out + 2 * i + 1);
    }
    if (turn_out) __builtin_nontemporal_store((uint8_t)t_out, turn_out + i);
    if (flips_out) __builtin_nontemporal_store(f, flips_out + i);
    if (ret_out) __builtin_nontemporal_store((int8_t)r, ret_out + i);
    if (nturn && r >= 0) nturn[i] = (uint8_t)(nturn[i] + 1);
}

constexpr int kStepPerThread = 1;
// kStepPerThread boards per thread, kBlock * gridDim apart (each load
// instruction still coalesced), all loaded before any is computed
__global__ __launch_bounds__(kBlock) void step_kernel(const u64* boards_in, const uint8_t* turn_in,
                                                      const uint8_t* __restrict__ move, u64* boards_out,
                                                      uint8_t* turn_out, u64* __restrict__ flips_out,
                                                      u64* __restrict__ legal_next, int8_t* __restrict__ ret_out,
                                                      uint8_t* __restrict__ nturn, int64_t n) {
    const int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x, stride = (int64_t)gridDim.x * kBlock;
    ulonglong2 b[kStepPerThread];
    u32 t[kStepPerThread], mvc[kStepPerThread];
#pragma unroll
    for (int j = 0; j < kStepPerThread; j++) {
        const int64_t i = i0 + j * stride;
        if (i < n) {
            b[j] = reinterpret_cast<const ulonglong2*>(boards_in)[i];
            t[j] = turn_in[i];
            mvc[j] = move[i];
            // all the loads in flight together: without this hipcc sinks the move
            // load into the valid-turn branch, a second dependent HBM round trip per wave
            asm volatile("" ::"v"(t[j]), "v"(mvc[j]));
        }
    }
#pragma unroll
    for (int j = 0; j < kStepPerThread; j++) {
        const int64_t i = i0 + j * stride;
        if (i < n) step_board(i, b[j], t[j], mvc[j], boards_out, turn_out, flips_out, legal_next, ret_out, nturn);
    }
}

// hands_for_direc (board.py:124-139) for any origin and any direction: the
// facade's put / is_puttable_at / hands_for_direc with coordinates Python
// wraps (board[y][x] with x = -1 is file h) or does not check at all.  The scan
// runs from the origin as given: step k = 1..8 along (dx, dy); a square
// holding the hostile piece extends the run, one holding the piece itself
// ends it (kept), anything else -- an off-board step included -- discards it.
// So from an off-board origin a ray exists only if its first step lands on
// the board, and a run of 8 hostile squares is kept without a closing piece
// (board.py:129's loop ends first).  The returned squares are always those of
// steps 1..count, so the count is the whole answer.  One thread per
// (origin, direction), eight steps of two bit tests: the facade's
// batch-of-one calls, not a throughput path.
__device__ __forceinline__ bool step_on_board(int64_t x, int64_t d, int k, int64_t& out) {
    int64_t t;
    // an overflowing coordinate is far off the board
    return !__builtin_mul_overflow(d, (int64_t)k, &t) && !__builtin_add_overflow(x, t, &out) && out >= 0 && out < 8;
}
__global__ __launch_bounds__(kBlock) void hands_kernel(const u64* __restrict__ own, const u64* __restrict__ hostile,
                                                       const int64_t* __restrict__ xs, const int64_t* __restrict__ ys,
                                                       const int64_t* __restrict__ dxs,
                                                       const int64_t* __restrict__ dys,
                                                       uint8_t* __restrict__ count, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const u64 mine = own[i], opp = hostile[i];
    const int64_t x = xs[i], y = ys[i], dx = dxs[i], dy = dys[i];
    int run = 0;
    for (int k = 1; k < 9; k++) {
        int64_t nx, ny;
        const bool on = step_on_board(x, dx, k, nx) && step_on_board(y, dy, k, ny);
        const u64 bit = on ? 1ull << (nx + 8 * ny) : 0ull;
        if (opp & bit) {
            run = k;  // (a zero direction revisits one square: board.py appends it again)
        } else {
            if (!(mine & bit)) run = 0;  // empty / other / off-board: discard
            break;                       // own piece: keep
        }
    }
    count[i] = (uint8_t)run;
}

__global__ __launch_bounds__(kBlock) void result_kernel(const u64* __restrict__ boards, uint8_t* __restrict__ nb,
                                                        uint8_t* __restrict__ nw, int8_t* __restrict__ diff,
                                                        uint8_t* __restrict__ terminal, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(boards)[i];
    const int cb = __popcll(b.x), cw = __popcll(b.y);
    if (nb) nb[i] = (uint8_t)cb;
    if (nw) nw[i] = (uint8_t)cw;
    if (diff) diff[i] = (int8_t)(cb - cw);
    if (terminal) terminal[i] = (moves(b.x, b.y) == 0 && moves(b.y, b.x) == 0) ? 1 : 0;
}

// ---------------------------------------------------------------------------
// rollout kernel: persistent waves (grid = resident capacity); each wave
// dequeues a batch of 64 game ids (ONE returning atomic on the caller's work
// word), plays the 64 games to terminal in lockstep -- a finished lane is
// masked off until the whole batch is done -- and dequeues again.  The
// hardware balances the batches; no refill code runs inside the ply loop
// (measured cheaper than per-lane refill, profiles/design_history_r01_r04.md §Rollout scheduling).
//
// The work word is the caller's (include/othello.h): 0 when the launch
// starts, and 0 again when it ends.  A launch of B batches on W waves makes
// exactly B + W dequeues (one per batch, one failing dequeue per wave), so the
// dequeue that draws ticket 64 * (B + W - 1) is the last one of the launch and
// its wave puts the word back to 0.  No reset runs on the stream, and a graph
// replay finds the word at 0 like an eager launch does.
// ---------------------------------------------------------------------------

struct RolloutArgs {
    const u64* start;
    const uint8_t* start_turn;
    u64 seed_state;
    u64 game_id0;
    int n_random;
    u64* final_boards;
    int8_t* diff;
    uint8_t* plies;
    uint8_t* moves;
    long long* hist;
    int64_t n;
    unsigned long long* work;  // the caller's work word (0 at start, left at 0)
    u64 last_ticket;           // 64 * (batches + waves - 1): the launch's last dequeue
    u32 coop_cap;              // 1-ply policies: 0 = per-lane choice (lane_choose; tests), else cooperative
    EvalWeights ew[2];         // OTH_POLICY_EVAL only: Black's table, White's table (runner: A's, B's)
    // GameRunner schedule (RUNNER kernels, oth_rollout_runner): random budgets
    // of players A and B (already capped at 10), the colour draw, A's colours
    u32 n_rand_a, n_rand_b;
    int swap;
    uint8_t* a_black;
    // the random policy's batch-tail hand-over (on by default; OTH_HANDOFF_K=0
    // in the environment turns it off): a fresh batch hands its games over to
    // the wave's LDS pool once no more than handoff_k lanes are still playing
    u32 handoff_k;
};

// Batch-tail compaction (shipped since round 5 in the random-policy kernel
// without move records; OTH_HANDOFF_K=0 in the environment turns it off at
// run time, tools/diag/handoff.patch removes it).  When at most handoff_k
// lanes of a fresh batch are still playing (a __ballot of the loop's live
// lanes, __popcll), the wave parks those games -- the whole lane state, 32 B
// -- in its LDS pool, compacted to the pool's top by mbcnt, and dequeues the
// next batch; once 64 games are parked they are played out as a batch of their
// own, and a wave that finds the queue empty plays out what it has parked.
constexpr u32 kHandoffK = 16;                       // the default K (env OTH_HANDOFF_K)
constexpr u32 kHandoffKMax = 16;                    // the pool's capacity allows K up to this
constexpr int kPoolCap = 64 + (int)kHandoffKMax;    // < 64 parked + at most K more per batch
struct Parked {
    u64 P, O;        // the side to move's discs, the other side's
    u32 state, inc;  // GameRng
    u32 g;           // game index in the launch
    u32 bits;        // b0 | passed << 1 | discs0 << 2 (7 bits) | npass << 9
};
static_assert(sizeof(Parked) == 32, "two 16-B LDS accesses per parked game");
constexpr u64 kParkedGame = ~0ull;

// Move records of the random policy (RECORD): a lane's record is one 128-byte
// row and the batch's 64 games are consecutive, so the wave's records are one
// contiguous 8 KB span.  They are built in LDS (row stride 132 bytes, 33
// dwords: a ply's byte stores from the 64 lanes fall in different banks) and
// written out after the batch by 16-byte stores, 1 KB per wave instruction.
// (The 1-ply policies keep their direct stores: their kernels are VALU-bound
// and hide them, 0.72 ms per 262,144 greedy games with or without records,
// while the 33 KB stage would halve their resident blocks: 0.83 ms with it,
// eval 1.17 -> 1.46 ms; tools/diag/record_policies.py.)
// Stored a byte per lane per ply straight to memory, the records' lines were
// written partially, again and again: 0.74-0.77 GB of HBM traffic per
// 262,144-game launch for 38 MB of output (profiles/r03_profile_summary.json).
constexpr int kRecStride = OTH_MOVES_STRIDE + 4;
constexpr int kRecWaveBytes = 64 * kRecStride;
constexpr size_t rec_stage_bytes(int policy, bool record) {
    return record && policy == OTH_POLICY_RANDOM ? (size_t)(kBlock / 64) * kRecWaveBytes : 0;
}

// the random loop's fill order (bitboard.hpp analyse): with the VOP3 logic,
// 7-8-9 leaves the fewest same-bank v_bitop3_b32 in its loop (tools/valu_mix.py)
constexpr int kRandomFillOrder = 789;
// occupancy floor of the rollout kernels (launch bounds): random and eval
// >= 4 waves/SIMD (<= 128 VGPRs); greedy 5 (<= 96 VGPRs; hipcc spills 13
// per-batch registers, none in the child loop): with the record change above,
// two streams 3.198 -> 3.24e10 env-steps/s and one stream 2.140 -> 2.116 ms
// per 1M-game launch against 4 waves (profiles/r06_notes.md §10; round 5,
// before the record change: +1.0% at two streams, a mixed result at one)
constexpr int rollout_waves_per_simd(int policy) { return policy == OTH_POLICY_GREEDY ? 5 : 4; }
template <int POLICY, bool RECORD, bool RUNNER = false>
__global__ __launch_bounds__(kBlock, rollout_waves_per_simd(POLICY)) void rollout_kernel(RolloutArgs a) {
    __shared__ unsigned long long hist_s[OTH_HIST_BINS];
    __shared__ uint8_t kth_tab[256 * 8];
    __shared__ u64 rays[kTabRows * 64];
    __shared__ int w_s[POLICY == OTH_POLICY_EVAL ? 2 * kEvalTable : 1];
    __shared__ CoopWave coop[POLICY == OTH_POLICY_RANDOM ? 1 : kBlock / 64];
    constexpr bool kPool = POLICY == OTH_POLICY_RANDOM && !RECORD && !RUNNER;
    __shared__ Parked pool_s[kPool ? kBlock / 64 : 1][kPool ? kPoolCap : 1];
    for (int k = threadIdx.x; k < OTH_HIST_BINS; k += kBlock) hist_s[k] = 0;
    kth_table_init(kth_tab);
    ray_table_init(rays);
    if (POLICY == OTH_POLICY_EVAL) {
        eval_weights_to_lds(a.ew[0], w_s);
        eval_weights_to_lds(a.ew[1], w_s + kEvalTable);
    }
    __syncthreads();

    const int lane = lane_id();
    const u64 n = (u64)a.n;
    u64 plies_sum = 0;
    constexpr bool kRecStage = RECORD && POLICY == OTH_POLICY_RANDOM;
    extern __shared__ u32 rec_dyn[];  // kRecStage: the block's waves' record stages
    uint8_t* const rec_wave = reinterpret_cast<uint8_t*>(rec_dyn) + (threadIdx.x >> 6) * kRecWaveBytes;
    uint8_t* const rec_row = rec_wave + lane * kRecStride;

    Parked* const pool = pool_s[kPool ? threadIdx.x >> 6 : 0];
    u32 parked = 0;          // wave-uniform: games in the wave's pool (kPool)
    bool exhausted = false;  // wave-uniform: the wave has made its failing dequeue
    (void)pool;
    (void)exhausted;
    for (;;) {
        // ---- dequeue a batch of 64 games (one per lane), or (kPool) take the
        // pool's parked games
        bool from_pool = false;
        u64 base = 0;
        if (kPool && parked >= 64u) {
            from_pool = true;
        } else if (!kPool || !exhausted) {
            if (lane == 0) {
                base = atomicAdd(a.work, 64ull);
                if (base == a.last_ticket) atomicExch(a.work, 0ull);  // every dequeue is done: reset
            }
            base = __shfl(base, 0);
            if (base >= n) {  // wave-uniform
                if (!kPool || parked == 0u) break;
                exhausted = true;
                from_pool = true;
            }
        } else {
            if (parked == 0u) break;
            from_pool = true;
        }

        u64 g = base + lane;
        bool active = !from_pool && g < n;
        u64 P = OPEN_BLACK, O = OPEN_WHITE;
        u32 side = OTH_BLACK, ply = 0;
        bool passed = false;
        GameRng rng;
        if (active) {
            rng.init(game_key(a.seed_state, a.game_id0 + g));
            if (a.start) {
                const ulonglong2 s0 = reinterpret_cast<const ulonglong2*>(a.start)[g];
                side = a.start_turn ? a.start_turn[g] : OTH_BLACK;
                side = side == OTH_WHITE ? OTH_WHITE : OTH_BLACK;
                P = side == OTH_BLACK ? s0.x : s0.y;
                O = side == OTH_BLACK ? s0.y : s0.x;
            }
            if (RECORD && !kRecStage) {
                uint4* mrec = reinterpret_cast<uint4*>(a.moves + g * OTH_MOVES_STRIDE);
#pragma unroll
                for (int q = 0; q < OTH_MOVES_STRIDE / 16; q++) mrec[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
            }
        }
        if constexpr (kRecStage) {  // the row starts 255-padded
#pragma unroll
            for (int q = 0; q < OTH_MOVES_STRIDE / 4; q++) reinterpret_cast<u32*>(rec_row)[q] = ~0u;
        }
        // a move code into game g's record (RECORD)
        auto rec_put = [&](u32 i, uint8_t code) {
            if (i >= OTH_MOVES_STRIDE) return;
            if constexpr (kRecStage) rec_row[i] = code;
            else a.moves[g * OTH_MOVES_STRIDE + i] = code;
        };

        // ---- play the batch: one env-step per active lane per iteration
        if constexpr (POLICY == OTH_POLICY_RANDOM) {
            // (kept separate: this exact loop is the measured config-3 kernel).  A
            // plain divergent loop: a lane leaves it with `break` at its terminal
            // and the loop runs while any lane is left, on the exec mask alone
            // (no per-iteration ballot).  The loop body is two plies, side0 to
            // move and then the other side (a pass also hands the move over), so
            // P stays side0's discs and O the other side's with no register
            // swap.  Without a move record the ply counter is not kept either:
            // every placement adds one disc, so plies = discs placed + passes
            // handed over (a pass just before the terminal is not an env-step).
            bool b0 = side == OTH_BLACK;
            u32 discs0 = RECORD ? 0u : (u32)__popcll(P | O);
            u32 npass = 0;  // passes (RECORD: every ply)
            if (kPool && from_pool) {  // the top (up to) 64 parked games
                const u32 take = min(parked, 64u);
                active = (u32)lane < take;
                if (active) {
                    const Parked e = pool[parked - take + lane];
                    P = e.P;
                    O = e.O;
                    rng.state = e.state;
                    rng.inc = e.inc;
                    g = e.g;
                    b0 = e.bits & 1u;
                    passed = (e.bits >> 1) & 1u;
                    discs0 = (e.bits >> 2) & 0x7fu;
                    npass = e.bits >> 9;
                }
                parked -= take;
            }
            const u32 hand_k = __builtin_amdgcn_readfirstlane(kPool && !from_pool ? a.handoff_k : 0u);
            const u32 parked0 = __builtin_amdgcn_readfirstlane(parked);
            (void)hand_k;
            (void)parked0;
            // one ply of mover X against Y; true at the terminal.  The
            // terminal's bookkeeping (final board, diff, plies, histogram) is
            // done once per lane after the loop, where P is still side0's
            // discs: inside it, the block ran whenever any lane of the wave
            // ended, ~7 times per batch.
            auto ply_of = [&](u64& X, u64& Y) -> bool {
                Position pos;
                analyse<kRandomFillOrder>(X, Y, pos);
                const u64 legal = pos.legal;
                // the move count serves the zero test and the pick
                const u32 c_lo = __popc((u32)legal), nl = c_lo + __popc((u32)(legal >> 32));
                if (nl == 0) {
                    // a full board is terminal at once: the other side has no
                    // empty square either, so the hand-over iteration (a
                    // second analysis) is skipped; 65% of random games end so
                    if (passed || (X | Y) == ~0ull) {
                        // terminal: both sides without a legal move (board.py:57-58);
                        // a pass handed over just before is not an env-step
                        if (passed) npass--;
                        return true;
                    }
                    // the mover must pass ('PS'): hand the move over
                    if (RECORD) rec_put(npass, OTH_PASS);
                    passed = true;
                    npass++;
                    return false;
                }
                passed = false;
                const u32 off = kth_bit_off(legal, rng.pick(nl), c_lo, kth_tab);
                const u64* col = ray_col(rays, off);
                const Flips f = flips_col(col[kRayRows * 64], run_sets(pos), col);
                if (RECORD) {
                    rec_put(npass, (uint8_t)(off >> 3));
                    npass++;
                }
                place(X, Y, f);
                return false;
            };
            if (active) {
                for (;;) {
                    if (ply_of(P, O)) break;
                    if (ply_of(O, P)) break;
                    if (kPool) {  // the batch's tail: park the lanes still playing
                        const u64 live = __ballot(1);
                        if ((u32)__popcll(live) <= hand_k) {
                            const u32 rank = __builtin_amdgcn_mbcnt_hi((u32)(live >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((u32)live, 0u));
                            pool[parked0 + rank] = Parked{P, O, rng.state, rng.inc, (u32)g,
                                                          (u32)b0 | (u32)passed << 1 | discs0 << 2 | npass << 9};
                            g = kParkedGame;
                            break;
                        }
                    }
                }
            }
            if (kPool) {
                const u64 pm = __ballot(active && g == kParkedGame);
                parked = parked0 + (u32)__popcll(pm);
                if (g == kParkedGame) active = false;
            }
            if (active) {
                const u32 ply = RECORD ? npass : (u32)__popcll(P | O) - discs0 + npass;
                if (RECORD) rec_put(ply, 0xFF);
                const u64 bl = b0 ? P : O, wh = b0 ? O : P;
                const int d = __popcll(bl) - __popcll(wh);
                if (a.final_boards) reinterpret_cast<ulonglong2*>(a.final_boards)[g] = make_ulonglong2(bl, wh);
                if (a.diff) a.diff[g] = (int8_t)d;
                if (a.plies) a.plies[g] = (uint8_t)ply;
                atomicAdd(&hist_s[d + 64], 1ull);
                atomicAdd(&hist_s[d > 0 ? 129 : (d < 0 ? 130 : 131)], 1ull);
                plies_sum += ply;
            }
        } else {
            // GameRunner schedule (RUNNER): the colour draw, then the random
            // budgets left by colour; tbl_black = the eval table Black plays
            u32 rem_b = 0, rem_w = 0, tbl_black = 0;
            if (RUNNER && active) {
                const bool ab = !(a.swap && rng.pick(2) == 1u);  // do_match's swap (subproc.py:28-32)
                rem_b = ab ? a.n_rand_a : a.n_rand_b;
                rem_w = ab ? a.n_rand_b : a.n_rand_a;
                tbl_black = ab ? 0u : 1u;
                if (a.a_black) a.a_black[g] = (uint8_t)ab;
            }
            while (__ballot(active)) {
                bool moving = false, choose = false;
                u32 sq = 0;
                Position pos;
                if (active) {
                    analyse(P, O, pos);
                    const u64 legal = pos.legal;
                    if (legal == 0) {
                        if (passed || (P | O) == ~0ull) {
                            // terminal: both sides without a legal move (board.py:57-58);
                            // a full board needs no hand-over iteration to know it
                            const u64 bl = side == OTH_BLACK ? P : O, wh = side == OTH_BLACK ? O : P;
                            const int d = __popcll(bl) - __popcll(wh);
                            // greedy (5 waves/SIMD, <= 96 VGPRs): the output
                            // addresses computed here from an opaque copy of g,
                            // and the game's plies into the block histogram
                            // directly, so that neither is a register live
                            // across the choice (hoisted, hipcc spilled them)
                            u64 gt = g;
                            if (POLICY == OTH_POLICY_GREEDY) asm volatile("" : "+v"(gt));
                            if (a.final_boards)
                                reinterpret_cast<ulonglong2*>(a.final_boards)[gt] = make_ulonglong2(bl, wh);
                            if (a.diff) a.diff[gt] = (int8_t)d;
                            if (a.plies) a.plies[gt] = (uint8_t)ply;
                            atomicAdd(&hist_s[d + 64], 1ull);
                            atomicAdd(&hist_s[d > 0 ? 129 : (d < 0 ? 130 : 131)], 1ull);
                            if (POLICY == OTH_POLICY_GREEDY) atomicAdd(&hist_s[132], (unsigned long long)ply);
                            else plies_sum += ply;
                            active = false;
                        } else {
                            // the mover must pass: hand the move over tentatively; the pass
                            // is counted once the other side turns out to have a move
                            passed = true;
                            const u64 t = P;
                            P = O;
                            O = t;
                            side ^= 3u;
                        }
                    } else {
                        if (passed) {
                            if (RECORD) rec_put(ply, OTH_PASS);
                            ply++;
                            passed = false;
                            if (RUNNER) {  // the passer's turn drew its coin (go_for, game_runner.py:134-135)
                                const u32 rx = side == OTH_BLACK ? rem_w : rem_b;
                                if (rx) (void)rng.pick(rx);
                            }
                        }
                        moving = true;
                        if (RUNNER) {
                            const u32 r = side == OTH_BLACK ? rem_b : rem_w;
                            if (r && rng.pick(r) == 0u) {  // go_for's coin: a random legal move (136-146)
                                sq = pick_legal(legal, rng, kth_tab);
                                if (side == OTH_BLACK) rem_b--;
                                else rem_w--;
                            } else {
                                choose = true;
                            }
                        } else if ((int)ply >= a.n_random) {
                            choose = true;  // decided below, by the whole wave
                        } else {
                            sq = pick_legal(legal, rng, kth_tab);
                        }
                    }
                }
                CoopWave& cw = coop[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)];  // wave-uniform: an SGPR base
                auto play = [&](u32 m, const RunSets& rs) {
                    if (RECORD) rec_put(ply, (uint8_t)m);
                    place(P, O, flips_rays(m, rs, rays));
                    const u64 np = O;
                    O = P;
                    P = np;
                    side ^= 3u;
                    ply++;
                };
                // Greedy (round 6): a move already decided (random) is played
                // before the wave's choice, a chosen one after it from the run
                // sets the lane published to its LDS record, so the position's
                // run sets are not live in VGPRs across every child of the
                // choice: greedy 2.152 -> 2.121 ms per 1M-game launch on one
                // stream, and room for 5 waves per SIMD (below).  Eval keeps
                // them in registers: the same change cost it 3.80 -> 3.97 ms
                // (tools/gpu_greedy_ab.sh, profiles/r06_notes.md).
                constexpr bool kFromRecord = POLICY == OTH_POLICY_GREEDY;
                if (kFromRecord && moving && !choose) play(sq, run_sets(pos));
                if (__ballot(choose)) {  // wave-uniform: every lane of the wave joins
                    const u32 tbl = side == OTH_BLACK ? tbl_black : tbl_black ^ 1u;
                    const u32 c = coop_choose<POLICY>(choose, P, O, tbl, pos, cw, rays, w_s, kth_tab, (u32)lane,
                                                      a.coop_cap);
                    if (choose) {
                        sq = c;
                        if (kFromRecord) {
                            u64 Pr, Or;
                            RunSets rs;
                            load_parent(cw.rec[lane], Pr, Or, rs);
                            play(c, rs);
                        }
                    }
                }
                if (!kFromRecord && moving) play(sq, run_sets(pos));
            }
        }
        if constexpr (kRecStage) {  // the wave's records, one contiguous span, 16 bytes a lane
            wave_sync();
            const int nvalid = (int)min<u64>(64, n - base);
            for (int c = lane; c < nvalid * (OTH_MOVES_STRIDE / 16); c += 64) {
                const int j = c / (OTH_MOVES_STRIDE / 16), part = c % (OTH_MOVES_STRIDE / 16);
                const u32* src = reinterpret_cast<const u32*>(rec_wave + j * kRecStride + part * 16);
                reinterpret_cast<uint4*>(a.moves + (base + j) * OTH_MOVES_STRIDE)[part] =
                    make_uint4(src[0], src[1], src[2], src[3]);
            }
            wave_sync();  // read out before the next batch pads the rows again
        }
    }

    // plies: wave reduction, one LDS atomic per wave
    for (int off = 32; off >= 1; off >>= 1) plies_sum += __shfl_xor(plies_sum, off);
    if (lane == 0) atomicAdd(&hist_s[132], (unsigned long long)plies_sum);
    __syncthreads();
    if (a.hist)
        for (int k = threadIdx.x; k < OTH_HIST_BINS; k += kBlock)
            if (hist_s[k]) atomicAdd((unsigned long long*)&a.hist[k], hist_s[k]);
}

// ---------------------------------------------------------------------------
// synthetic mid-game generator (config 2 inputs)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void sample_midgame_kernel(u64 S, u64 index0, u64* __restrict__ boards,
                                                                uint8_t* __restrict__ turn,
                                                                uint8_t* __restrict__ nturn,
                                                                uint8_t* __restrict__ move, int64_t n) {
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    const u64 i = index0 + (u64)j;
    for (u64 attempt = 0;; attempt++) {
        GameRng rng;
        rng.init(game_key(S, i ^ (attempt << 48)));
        const u32 target = 10 + rng.pick(40);  // the first draw picks the stopping ply
        u64 P = OPEN_BLACK, O = OPEN_WHITE;
        u32 side = OTH_BLACK, ply = 0;
        for (;;) {
            const u64 legal = moves(P, O);
            if (legal == 0 && moves(O, P) == 0) break;  // is_game_over
            if (ply >= target && legal) {
                const u32 sq = kth_bit(legal, rng.pick((u32)__popcll(legal)));
                reinterpret_cast<ulonglong2*>(boards)[j] =
                    side == OTH_BLACK ? make_ulonglong2(P, O) : make_ulonglong2(O, P);
                turn[j] = (uint8_t)side;
                if (nturn) nturn[j] = (uint8_t)ply;
                move[j] = (uint8_t)sq;
                return;
            }
            if (legal) {
                const u32 sq = kth_bit(legal, rng.pick((u32)__popcll(legal)));
                const u64 mv = 1ull << sq;
                const u64 f = flips_carry(sq, P, O);
                P = or3(P, f, mv);
                O = andn(O, f);
            }
            const u64 t = P;
            P = O;
            O = t;
            side ^= 3u;
            ply++;
        }
    }
}

// ---------------------------------------------------------------------------
// §8f row 1: book emitter.  Replay recorded move codes into every recorded
// position (game_runner.py:169-184 records the board after Board() and after
// every put_s), with is_game_over per position (game_recorder.py:107-114).
// ---------------------------------------------------------------------------
// One lane per game; HBM traffic is kept to the bytes the ABI defines:
//  * board rows: a lane's rows are its own (stride OTH_POS_STRIDE), so one
//    store instruction touches 64 different lines.  Positions are buffered
//    8 at a time, and the bursts are aligned so that each one fills exactly
//    one 128-B line (row i*129 + p starts a line when (i + p) % 8 == 0, since
//    129 = 1 mod 8): every line is written whole by 8 back-to-back stores
//    instead of lingering half-written in L2 (one store per position let
//    partial lines be evicted: 3.4 GB of traffic per 262,144-game launch for
//    0.64 GB of output);
//  * move codes: the lane's 128-B record is read once, by 8 dwordx4 loads, into
//    a register shift register (a byte load per position re-fetched lines the
//    L2 had evicted in between);
//  * turn / end bytes: staged in LDS as one packed byte per position (turn in
//    bits 0-6, is_game_over in bit 7) at the block's own output layout, then
//    written out as the block's two contiguous ranges by coalesced 16-B stores
//    (per-lane byte stores at stride 129 touched a line per lane per position).
//    Rows past plies are written as 0.  A turn >= 127 can only be the game's
//    start turn (put_s sets the turn to Black or White), so it is staged as the
//    escape 127 and restored from start_turn on the way out.
constexpr int kReplayBurst = 8;                         // positions per burst: one 128-B line of rows
constexpr int kReplayStage = kBlock * OTH_POS_STRIDE;  // packed turn/end bytes of one block
constexpr u32 kTurnEscape = 0x7f;
static_assert(kReplayStage % 16 == 0, "block stage = whole 16-B chunks");

__device__ __forceinline__ void load_move_record(const uint8_t* row, bool vec, u64 (&R)[OTH_MOVES_STRIDE / 8]) {
    if (vec) {
        const ulonglong2* r2 = reinterpret_cast<const ulonglong2*>(row);
#pragma unroll
        for (int j = 0; j < OTH_MOVES_STRIDE / 16; j++) {
            const ulonglong2 v = r2[j];
            R[2 * j] = v.x;
            R[2 * j + 1] = v.y;
        }
    } else {  // a caller's record that is not 16-B aligned
#pragma unroll
        for (int j = 0; j < OTH_MOVES_STRIDE / 8; j++) {
            u64 w = 0;
#pragma unroll 1
            for (int k = 0; k < 8; k++) w |= (u64)row[8 * j + k] << (8 * k);
            R[j] = w;
        }
    }
}

// The bursts go out through a per-wave LDS exchange: after a lane has built
// half a burst (4 rows = 64 B of one line), the wave's 64 half-lines are
// stored by 4 lanes each, so a store instruction writes 16 half-lines of 64
// contiguous bytes instead of 64 scattered 16-B rows.
constexpr int kReplayBursts = (OTH_POS_STRIDE + 7 + kReplayBurst - 1) / kReplayBurst;  // 17 for every alignment
constexpr int kXHalf = kReplayBurst / 2;  // rows per exchange
// the packed layout's stage: the block's bytes start at a 16-B chunk offset of
// up to 15, and its turn / end ranges are chunked from there.  Sized for 72
// rows per game (round 6; self-play games record 61-62 rows on average and
// at most ~70), not the stride's 129: a block whose rows do not fit writes its
// bytes directly (below).  With the 16 KiB row exchange that is 37 KiB of LDS
// per block, so 4 blocks fit a CU, and the 4,096 waves of a 262,144-game launch
// are resident at once instead of in one and a third rounds.
constexpr int kReplayPackedRows = 72;
constexpr int kReplayStagePacked = kBlock * kReplayPackedRows + 16;

// Two output layouts (include/othello.h):
//  * strided (PACKED = false): game i's position p at row i*OTH_POS_STRIDE + p,
//    every row of the stride written (rows past plies as 0);
//  * packed (PACKED = true, oth_replay_rows): game i's position p at row
//    row_off[i] + p, only rows p <= plies written: the useful bytes alone.
//    A wave runs only as many bursts as its longest game needs (the strided
//    layout runs all 17 to zero the rest of the stride), and the block's turn
//    / end bytes are one contiguous range starting anywhere, staged from its
//    16-B chunk boundary; the chunks the range shares with the neighbouring
//    blocks are written byte by byte.
template <bool PACKED>
__global__ __launch_bounds__(kBlock, PACKED ? 4 : 3) void replay_kernel(const u64* __restrict__ start,
                                                        const uint8_t* __restrict__ start_turn,
                                                        const uint8_t* __restrict__ moves,
                                                        const uint8_t* __restrict__ plies,
                                                        const int64_t* __restrict__ row_off, u64* __restrict__ pos,
                                                        uint8_t* __restrict__ pos_turn, uint8_t* __restrict__ pos_end,
                                                        int64_t n, int vec_moves, int vec_out) {
    extern __shared__ uint4 replay_stage4[];  // the block's packed turn/end bytes when turn or end is wanted
    __shared__ uint4 xrow[kBlock * kXHalf];   // lane-major: lane's 4 rows
    __shared__ unsigned long long xaddr[kBlock];
    __shared__ u32 xmask[kBlock];
    uint8_t* stage = reinterpret_cast<uint8_t*>(replay_stage4);
    const bool staged = pos_turn || pos_end;
    const int64_t blk0 = (int64_t)blockIdx.x * kBlock;
    const int nb = (int)min<int64_t>(kBlock, n - blk0);
    const int lane = threadIdx.x;
    const int wl = lane & 63, wbase = lane & ~63;
    // the block's output rows [base, base + bytes) and (packed) the 16-B chunk
    // they start in.  Packed: the lowest first row and the highest end over the
    // block's games (the first game's row and the last game's end for the
    // prefix-sum offsets the header asks for).  With other offsets a block
    // whose rows do not fit the LDS stage writes its bytes directly (and a gap
    // between games is left as the caller had it); taken over every game, not
    // only the last, no game's stage pointer can leave the stage.
    int64_t base = blk0 * OTH_POS_STRIDE, bytes = (int64_t)nb * OTH_POS_STRIDE;
    if (PACKED && staged) {
        __shared__ long long rows_lo[kBlock / 64], rows_hi[kBlock / 64];
        long long lo = LLONG_MAX, hi = LLONG_MIN;
        if (threadIdx.x < nb) {
            lo = row_off[blk0 + threadIdx.x];
            hi = lo + min<int>(plies[blk0 + threadIdx.x], OTH_MOVES_STRIDE) + 1;
        }
        for (int off = 32; off >= 1; off >>= 1) {
            lo = min(lo, __shfl_xor(lo, off));
            hi = max(hi, __shfl_xor(hi, off));
        }
        if ((threadIdx.x & 63) == 0) {
            rows_lo[threadIdx.x >> 6] = lo;
            rows_hi[threadIdx.x >> 6] = hi;
        }
        __syncthreads();
        for (int w = 0; w < kBlock / 64; w++) {
            lo = min(lo, rows_lo[w]);
            hi = max(hi, rows_hi[w]);
        }
        base = lo;
        bytes = hi - lo;
    } else if (PACKED) {
        base = row_off[blk0];
    }
    const int64_t base_al = PACKED ? (base & ~(int64_t)15) : base;
    const int lead = (int)(base - base_al);  // stage bytes before the block's first (packed only)
    const int64_t span = lead + bytes;
    const bool direct = PACKED && staged && span > kReplayStagePacked;
    if (staged && !direct) {  // rows past plies (strided) and any gap (packed) are staged as 0
        for (int c = lane; c < (PACKED ? kReplayStagePacked : kReplayStage) / 16; c += kBlock)
            replay_stage4[c] = make_uint4(0, 0, 0, 0);
        __syncthreads();
    }
    // every lane of a wave runs the wave's bursts (the exchange is wave-wide);
    // a lane past the launch's last game has nothing valid to store
    const bool live = lane < nb;
    const int64_t i = blk0 + (live ? lane : 0);
    u64 bl = OPEN_BLACK, wh = OPEN_WHITE;
    u32 t = OTH_BLACK;
    if (live && start) {
        const ulonglong2 s0 = reinterpret_cast<const ulonglong2*>(start)[i];
        bl = s0.x;
        wh = s0.y;
        t = start_turn ? start_turn[i] : OTH_BLACK;
    }
    const int np = live ? min<int>(plies[i], OTH_MOVES_STRIDE) : -1;
    u64 R[OTH_MOVES_STRIDE / 8];
    if (live) load_move_record(moves + i * OTH_MOVES_STRIDE, vec_moves != 0, R);
    else
#pragma unroll
        for (int j = 0; j < OTH_MOVES_STRIDE / 8; j++) R[j] = 0;
    const int64_t row0 = PACKED ? (live ? row_off[i] : base) : i * OTH_POS_STRIDE;
    ulonglong2* out = reinterpret_cast<ulonglong2*>(pos) + row0;
    uint8_t* st = stage + (direct ? 0 : row0 - base_al);
    // the packed turn/end byte of position p: to the stage, or (direct) unpacked
    // straight to the outputs (the start turn is then written as it is)
    auto put_te = [&](int p, u32 v, u32 t_full) {
        if (!direct) {
            st[p] = (uint8_t)v;
        } else {
            if (pos_turn) pos_turn[row0 + p] = (uint8_t)t_full;
            if (pos_end) pos_end[row0 + p] = (uint8_t)(v >> 7);
        }
    };
    const int s = (int)(row0 & 7);  // the first burst starts at p = -s: whole lines from there on
    // bursts this wave runs: all 17 (strided), or enough for its longest game
    int bursts = kReplayBursts;
    if (PACKED) {
        bursts = live ? (np + 1 + s + kReplayBurst - 1) / kReplayBurst : 0;
        for (int off = 32; off >= 1; off >>= 1) bursts = max(bursts, __shfl_xor(bursts, off));
    }
    u64 prev = 0, cur = R[0];   // move-record words w[b-1], w[b] of burst b
    for (int bi = 0; bi < bursts; bi++) {
        const int p0 = 8 * bi - s;
        // move codes p0 .. p0+7 (bytes before position 0 are never used)
        const u64 win = s ? (cur << (8 * s)) | (prev >> (64 - 8 * s)) : cur;
        // each half's 4 rows go straight into the wave's LDS exchange as they
        // are built (round 6: an 8-row register buffer held 32 more VGPRs)
#pragma unroll
        for (int h = 0; h < kReplayBurst / kXHalf; h++) {
          u32 valid = 0;
#pragma unroll
          for (int kk = 0; kk < kXHalf; kk++) {
            const int k = h * kXHalf + kk;
            const int p = p0 + k;
            ulonglong2 row = make_ulonglong2(0ull, 0ull);  // rows past plies are 0
            if (p >= 0 && p <= np) {
                row = make_ulonglong2(bl, wh);
                const u32 c = (u32)(win >> (8 * k)) & 0xffu;
                const bool fast = t == OTH_BLACK || t == OTH_WHITE;
                if (pos_end && fast) {
                    // A recorded move that flips proves the mover can move, so
                    // the position is not over and only the move's flips are
                    // needed (flips_carry, ~85 VALU); a pass, an illegal code or
                    // the last position takes is_game_over the long way (an
                    // analysis, and the other side's only where the mover has
                    // no move).  One analysis for both, with the flips from its
                    // run sets, cost ~165 VALU at every position.
                    const bool black = t == OTH_BLACK;
                    u64 P = black ? bl : wh, O = black ? wh : bl;
                    u64 f = 0;
                    if (p < np && c < 64 && !((P | O) >> c & 1ull)) f = flips_carry(c, P, O);
                    u32 e = 0;
                    if (!f && moves_of(P, O) == 0) e = moves_of(O, P) == 0;
                    put_te(p, t | (e << 7), t);
                    if (f) {
                        P = or3(P, f, 1ull << c);
                        O = andn(O, f);
                        bl = black ? P : O;
                        wh = black ? O : P;
                        t ^= 3u;
                    } else if (p < np && c == OTH_PASS) {
                        t ^= 3u;
                    }
                } else {
                if (staged) {
                    u32 e = 0;
                    if (pos_end && moves_of(bl, wh) == 0) e = moves_of(wh, bl) == 0;
                    put_te(p, min(t, kTurnEscape) | (e << 7), t);
                }
                // put_s semantics (board.py:192-209): pass toggles; illegal leaves the state
                if (p < np && !fast) {
                    const StepOut o = put_s_any(bl, wh, t, c);  // side Empty / none (rare)
                    bl = o.bl;
                    wh = o.wh;
                    t = o.t;
                } else if (p < np) {
                    if (c == OTH_PASS) {
                        t ^= 3u;
                    } else if (c < 64) {
                        const bool black = t == OTH_BLACK;
                        u64 P = black ? bl : wh, O = black ? wh : bl;
                        const u64 mm = 1ull << c;
                        if (!((P | O) & mm)) {
                            const u64 f = flips_carry(c, P, O);
                            if (f) {
                                P |= f | mm;
                                O = andn(O, f);
                                bl = black ? P : O;
                                wh = black ? O : P;
                                t ^= 3u;
                            }
                        }
                    }
                }
                }
            }
            xrow[lane * kXHalf + kk] = make_uint4((u32)row.x, (u32)(row.x >> 32), (u32)row.y, (u32)(row.y >> 32));
            valid |= (live && p >= 0 && p < (PACKED ? np + 1 : OTH_POS_STRIDE) ? 1u : 0u) << kk;
          }
            xaddr[lane] = reinterpret_cast<unsigned long long>(out + (p0 + h * kXHalf));
            xmask[lane] = valid;
            wave_sync();
#pragma unroll
            for (int j = 0; j < 64 / (64 / kXHalf); j++) {
                const int src = wbase + j * (64 / kXHalf) + wl / kXHalf, c = wl % kXHalf;
                if (xmask[src] >> c & 1u)
                    reinterpret_cast<uint4*>(xaddr[src])[c] = xrow[src * kXHalf + c];
            }
            wave_sync();  // the wave has read this half before the next overwrites it
        }
        prev = cur;
#pragma unroll
        for (int j = 0; j < OTH_MOVES_STRIDE / 8 - 1; j++) R[j] = R[j + 1];
        R[OTH_MOVES_STRIDE / 8 - 1] = 0;
        cur = R[0];
    }
    if (!staged || direct) return;
    __syncthreads();
    // the block's rows of pos_turn / pos_end are one contiguous range each:
    // global bytes [base, base + bytes), staged from base_al
    // the game of a staged byte (the escape path only): by division, or by a
    // linear scan of the block's games for the one whose rows
    // [row_off, row_off + plies] hold it.  The offsets of a staged block need
    // not increase (any disjoint layout stages), so no binary search; an
    // escaped byte is rare (a start turn >= 127 still to move) and a block has
    // at most 256 games.  Escape bytes are only ever staged for a game's own
    // rows, so the scan always finds one.
    auto game_of = [&](int64_t q) -> int64_t {
        if (!PACKED) return blk0 + q / OTH_POS_STRIDE;
        const int64_t row = base_al + q;
        for (int k = 0; k < nb; k++) {
            const int64_t r0 = row_off[blk0 + k];
            if (row >= r0 && row <= r0 + min<int>(plies[blk0 + k], OTH_MOVES_STRIDE)) return blk0 + k;
        }
        return blk0;
    };
    if (vec_out) {
        for (int c = lane; c * 16 < span; c += kBlock) {
            const uint4 v = replay_stage4[c];
            u32 w[4] = {v.x, v.y, v.z, v.w};
            u32 tw[4], ew[4];
            bool esc = false;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                tw[q] = w[q] & 0x7f7f7f7fu;
                ew[q] = (w[q] >> 7) & 0x01010101u;
                esc |= ((tw[q] + 0x01010101u) & 0x80808080u) != 0;  // a byte == 0x7f
            }
            const int64_t q0 = (int64_t)c * 16;
            if (esc) {  // rare: a start turn >= 127 still to move
#pragma unroll 1
                for (int q = 0; q < 16; q++) {
                    if (q0 + q < lead || q0 + q >= span) continue;
                    const u32 byte = w[q >> 2] >> (8 * (q & 3)) & 0xffu;
                    if ((byte & kTurnEscape) != kTurnEscape) continue;
                    const u32 tb = start_turn[game_of(q0 + q)];
                    tw[q >> 2] = (tw[q >> 2] & ~(0xffu << (8 * (q & 3)))) | (tb << (8 * (q & 3)));
                }
            }
            const int64_t g0 = base_al + q0;  // global byte of the chunk's first
            if (q0 >= lead && q0 + 16 <= span) {
                if (pos_turn) *reinterpret_cast<uint4*>(pos_turn + g0) = make_uint4(tw[0], tw[1], tw[2], tw[3]);
                if (pos_end) *reinterpret_cast<uint4*>(pos_end + g0) = make_uint4(ew[0], ew[1], ew[2], ew[3]);
            } else {  // a chunk the range shares with a neighbour, or the launch's last
                for (int q = 0; q < 16; q++) {
                    if (q0 + q < lead || q0 + q >= span) continue;
                    if (pos_turn) pos_turn[g0 + q] = (uint8_t)(tw[q >> 2] >> (8 * (q & 3)));
                    if (pos_end) pos_end[g0 + q] = (uint8_t)(ew[q >> 2] >> (8 * (q & 3)));
                }
            }
        }
    } else {  // a caller's output that is not 16-B aligned: coalesced byte stores
        for (int64_t o = lead + lane; o < span; o += kBlock) {
            const u32 c = stage[o];
            // only an escaped turn needs its game (a search of the row offsets)
            const uint8_t tb = (c & kTurnEscape) == kTurnEscape ? start_turn[game_of(o)] : (uint8_t)(c & kTurnEscape);
            if (pos_turn) pos_turn[base_al + o] = tb;
            if (pos_end) pos_end[base_al + o] = (uint8_t)(c >> 7);
        }
    }
}

// serialize_str (board.py:214-243) + '\n' of record r = 67 bytes: 64 squares
// row-major ('O' black, 'X' white, '-' empty), ' ', the side ('O' / 'X' /
// '-'), '\n'.  One lane per line: a rank of 8 squares becomes 8 characters
// at once from a byte-expansion table (byte k of kExpand[b] is 0xFF iff bit k
// of b is set), and the wave's 64 lines (4,288 contiguous bytes) are
// assembled in LDS -- each lane ORs its line in at its byte offset, the two
// dwords it shares with its neighbours included -- and stored by the whole
// wave as aligned 16-byte chunks.  (The first version had every lane build
// 16 bytes of text character by character, ~8 VALU each: 1.85 TB/s.)
constexpr int kLine = 67;
constexpr int kBookWave = 64 * kLine;  // 4,288 = 268 x 16 bytes
__device__ __forceinline__ u64 rank_chars(u64 bl, u64 wh, u32 rank, const u64* ex) {
    const u64 mb = ex[(u32)(bl >> (8 * rank)) & 0xFFu], mw = ex[(u32)(wh >> (8 * rank)) & 0xFFu];
    // '-' ^ ('O' ^ '-') on Black squares ^ ('X' ^ '-') on White ones
    return 0x2D2D2D2D2D2D2D2Dull ^ (mb & 0x6262626262626262ull) ^ (mw & 0x7575757575757575ull);
}
__global__ __launch_bounds__(kBlock) void book_text_kernel(const u64* __restrict__ boards,
                                                           const uint8_t* __restrict__ turn, int64_t n,
                                                           uint8_t* __restrict__ out, int vec_out) {
    __shared__ u64 ex[256];
    __shared__ u32 stage_all[(kBlock / 64) * (kBookWave / 4)];
    for (int e = threadIdx.x; e < 256; e += kBlock) {
        u64 m = 0;
        for (int k = 0; k < 8; k++)
            if (e >> k & 1) m |= 0xFFull << (8 * k);
        ex[e] = m;
    }
    const int wl = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32* st = stage_all + wv * (kBookWave / 4);
    for (int d = wl; d < kBookWave / 4; d += 64) st[d] = 0;
    __syncthreads();
    const int64_t line0 = ((int64_t)blockIdx.x * (kBlock / 64) + wv) * 64;  // the wave's first line
    const int64_t li = line0 + wl;
    if (li < n) {
        const ulonglong2 b = reinterpret_cast<const ulonglong2*>(boards)[li];
        const u32 t = turn[li];
        // the line as 17 dwords (the 17th: ' ', side, '\n')
        u32 L[18];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u64 w = rank_chars(b.x, b.y, (u32)r, ex);
            L[2 * r] = (u32)w;
            L[2 * r + 1] = (u32)(w >> 32);
        }
        const u32 side = t == OTH_BLACK ? 'O' : (t == OTH_WHITE ? 'X' : '-');
        L[16] = 0x20u | (side << 8) | (0x0Au << 16);
        L[17] = 0;
        // byte offset 67 * wl = 4 * d0 + phi: dword k of the shifted line is
        // bytes [4k - phi, 4k - phi + 4) of the line
        const u32 o = (u32)wl * kLine, d0 = o >> 2, sh = 8u * (o & 3u);
        u32 lo = 0;
#pragma unroll
        for (int k = 0; k < 18; k++) {
            const u32 v = (u32)((((u64)L[k] << 32) | lo) >> (32 - sh));
            lo = L[k];
            // the first and the last dword are shared with the neighbouring
            // lines (bytes outside this line are 0 here): OR them in
            if (k == 0 || k >= 16) {
                if (v) atomicOr(&st[d0 + k], v);
            } else {
                st[d0 + k] = v;
            }
        }
    }
    wave_sync();
    const int64_t bytes = (min<int64_t>(n, line0 + 64) - line0) * kLine;
    if (bytes <= 0) return;
    uint8_t* dst = out + line0 * kLine;  // line0 * 67 is a multiple of 16 (line0 is of 64)
    for (int c = wl; c * 16 < bytes; c += 64) {
        const uint4 v = reinterpret_cast<const uint4*>(st)[c];
        if (vec_out && c * 16 + 16 <= bytes) {
            *reinterpret_cast<uint4*>(dst + c * 16) = v;
        } else {  // the launch's last partial chunk, or a caller's output that is not 16-B aligned
            const u32 w[4] = {v.x, v.y, v.z, v.w};
            for (int q = 0; q < 16 && c * 16 + q < bytes; q++) dst[c * 16 + q] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
        }
    }
}

// Book ingest: the reader's side of the same format (game_reader.py,
// replearn.learn_books) -- board strings back into bitboards, one lane per
// string.  Four characters at a time: the bytes of a dword equal to 'O' (or
// 'X') are found with the exact zero-byte test (t = w ^ "OOOO": a byte of t is
// zero iff its high bit stays clear in ((t & 0x7F..) + 0x7F..) | t), and their
// four flags are gathered into four consecutive bits.
__device__ __forceinline__ u32 chars_eq4(u32 w, u32 c4) {
    const u32 t = w ^ c4;
    const u32 q = (~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u) >> 7;  // bits 0, 8, 16, 24
    return (q | (q >> 7) | (q >> 14) | (q >> 21)) & 0xFu;
}
__device__ __forceinline__ u32 side_of_char(u32 c) { return c == 'O' ? OTH_BLACK : (c == 'X' ? OTH_WHITE : 0u); }
// Strings at a stride that is not a multiple of 16 (the 67-byte lines of a
// flat file) are read byte by byte: 4.1 TB/s over the lines of 262,144 games.
// Measured slower: staging each wave's 64-line span through LDS with 16-B
// loads and funnel-shifting each lane's 17 dwords out of it (the mirror of
// book_text_kernel's exchange), 3.6 TB/s; the lane's 17 covering dwords
// loaded straight from memory and funnel-shifted, 3.2-3.3 TB/s.
__global__ __launch_bounds__(kBlock) void book_parse_kernel(const uint8_t* __restrict__ text, int64_t stride,
                                                            u64* __restrict__ boards, uint8_t* __restrict__ turn,
                                                            int64_t n, int vec) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint8_t* s = text + i * stride;
    u32 w[16];
    if (vec) {  // 16-B aligned strings: four dwordx4 loads
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 v = reinterpret_cast<const uint4*>(s)[q];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++)
            w[k] = (u32)s[4 * k] | (u32)s[4 * k + 1] << 8 | (u32)s[4 * k + 2] << 16 | (u32)s[4 * k + 3] << 24;
    }
    u32 b[2] = {0, 0}, x[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++) {
        b[k >> 3] |= chars_eq4(w[k], 0x4F4F4F4Fu) << (4 * (k & 7));  // 'O'
        x[k >> 3] |= chars_eq4(w[k], 0x58585858u) << (4 * (k & 7));  // 'X'
    }
    reinterpret_cast<ulonglong2*>(boards)[i] =
        make_ulonglong2(((u64)b[1] << 32) | b[0], ((u64)x[1] << 32) | x[0]);
    if (turn) turn[i] = (uint8_t)side_of_char(s[65]);
}

// ---------------------------------------------------------------------------
// §8f row 2: learner features, counts() of parameter_progress_position_moves_learn.py:5-17:
// (64 - n_empty, n_puttable_for(side), mask_count(side, m) for the 8 region masks)
// ---------------------------------------------------------------------------
// counts()' view of a board for a side code: 1/2 = 'O'/'X'; 0 = any other
// side string (turn_from_string -> Empty: mask_count counts empty squares and
// the mobility is puttables(Empty)); >= 3 has no reference string and matches
// nothing (mask counts 0, mobility 0, as board.py would for that piece value)
__device__ __forceinline__ void side_view(ulonglong2 b, u32 sd, u64& mine, u64& mob) {
    if (sd == OTH_BLACK || sd == OTH_WHITE) {
        mine = sd == OTH_BLACK ? b.x : b.y;
        mob = moves_of(mine, sd == OTH_BLACK ? b.y : b.x);
    } else if (sd == 0) {
        mine = ~(b.x | b.y);
        mob = moves_empty_side(b.x, b.y);
    } else {
        mine = 0;
        mob = 0;
    }
}

__global__ __launch_bounds__(kBlock) void features_kernel(const u64* __restrict__ boards,
                                                          const uint8_t* __restrict__ side,
                                                          uint8_t* __restrict__ out, int64_t n) {
    // (an LDS-assembled, 16-byte-store variant of the 10-byte rows measured
    // slower, 226 against 206 us over 33.8M positions: the kernel is bound by
    // its analysis per position, not by the byte stores)
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(boards)[i];
    u64 mine, mob;
    side_view(b, side[i], mine, mob);
    uint8_t* o = out + i * OTH_FEATURES;
    o[0] = (uint8_t)__popcll(b.x | b.y);
    o[1] = (uint8_t)__popcll(mob);
#pragma unroll
    for (int k = 0; k < 8; k++) o[2 + k] = (uint8_t)__popcll(mine & kRegionMasks[k]);
}

// oth_eval: the linear eval of each position from side[i]'s view (features as
// features_kernel, side codes as side_view)
__global__ __launch_bounds__(kBlock) void eval_kernel(const u64* __restrict__ boards, const uint8_t* __restrict__ side,
                                                      EvalWeights ew, int32_t* __restrict__ out, int64_t n) {
    __shared__ int w_s[OTH_EVAL_PHASES * kEvalRow];
    eval_weights_to_lds(ew, w_s);
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(boards)[i];
    u64 mine, mob;
    side_view(b, side[i], mine, mob);
    const int* w = w_s + kEvalRow * eval_shard((u32)__popcll(b.x | b.y));
    out[i] = eval_linear(w, mine, mob);
}

// ---------------------------------------------------------------------------
// TD state map (progress_position_moves_learn.py:37-62), include/othello.h
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t td_key(ulonglong2 b, u32 sd) {
    u64 mine, mob;
    side_view(b, sd, mine, mob);
    // include/othello.h OTH_TD_KEY_BITS layout
    constexpr int kShift[8] = {27, 23, 20, 16, 12, 7, 4, 0};
    u64 k = ((u64)__popcll(b.x | b.y) << 36) | ((u64)__popcll(mob) << 30);
#pragma unroll
    for (int r = 0; r < 8; r++) k |= (u64)__popcll(mine & kRegionMasks[r]) << kShift[r];
    return (int64_t)k;
}
// the same counts() as the packed words' sort key (td_skey.hpp)
__device__ __forceinline__ u64 td_skey_of(ulonglong2 b, u32 sd) {
    u64 mine, mob;
    side_view(b, sd, mine, mob);
    u32 r[8];
#pragma unroll
    for (int k = 0; k < 8; k++) r[k] = (u32)__popcll(mine & kRegionMasks[k]);
    return td_skey::encode((u32)__popcll(b.x | b.y), (u32)__popcll(mob), r);
}

// The same updates, one wave per game (round 5): lane p takes the game's
// positions p, p + 64, ... .  One thread per (g, p) slot of the 129-row stride
// leaves about half the lanes of the waves that do work idle (a game records
// ~62 positions of its 129 slots, and the waves straddle games); here a wave
// idles only on the lanes past the game's own positions.  The game's plies,
// row offset, base and terminal row are wave-uniform (scalar loads).  A wave
// takes kTdUpdGames = 4 games (late round 5): 195 -> 177 us per 32.2M
// updates (1: 195, 2: 179-183, 8: 175-177 at 112 VGPRs; tools/diag/td_ab.sh).
// (The round-4 kernel, one thread per (g, p) slot: tools/diag/r05_variants.patch.)
// kTdUpdGames games per wave, one after the other: their scalar loads
// (plies, row offset, base, terminal row) and first-round row loads are issued
// before any game's words are computed, so a wave waits on one dependent
// chain of loads for all of them instead of one chain per game.
constexpr int kTdUpdGames = 4;
// the words (or key/value pairs) of position p of a game whose terminal
// position np gives value_for_black vb; first update index jb
template <bool WORDS>
__device__ __forceinline__ void td_update_pair(ulonglong2 b, u32 p, u32 np, int vb, int64_t jb,
                                               const double* __restrict__ lam_pow, int64_t* __restrict__ keys,
                                               double* __restrict__ vals, u64* __restrict__ words) {
    const int64_t j = jb + 2 * (int64_t)(np - p);
    if (WORDS) {
        const u64 t = (u64)(np - p) << OTH_TD_PACK_TURN_SHIFT;
        words[j] = ((u64)(vb + 64) << OTH_TD_PACK_VALUE_SHIFT) | t | td_skey_of(b, OTH_BLACK);
        words[j + 1] = ((u64)(64 - vb) << OTH_TD_PACK_VALUE_SHIFT) | t | td_skey_of(b, OTH_WHITE);
        return;
    }
    const double lam = lam_pow[np - p];
    keys[j] = td_key(b, OTH_BLACK);
    vals[j] = (double)vb * lam;
    keys[j + 1] = td_key(b, OTH_WHITE);
    vals[j + 1] = (double)(-vb) * lam;
}
template <bool WORDS>
__global__ __launch_bounds__(kBlock) void td_updates_wave_kernel(const u64* __restrict__ pos,
                                                                 const int64_t* __restrict__ row_off,
                                                                 const uint8_t* __restrict__ plies,
                                                                 const int64_t* __restrict__ base,
                                                                 const double* __restrict__ lam_pow,
                                                                 int64_t* __restrict__ keys, double* __restrict__ vals,
                                                                 u64* __restrict__ words, int64_t n) {
    constexpr int G = kTdUpdGames;
    const int64_t g0 =
        ((int64_t)blockIdx.x * (kBlock / 64) + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))) * G;
    if (g0 >= n) return;
    const u32 lane = threadIdx.x & 63u;
    const int ng = (int)min<int64_t>(G, n - g0);  // wave-uniform
    u32 np[G];
    const ulonglong2* row[G];
#pragma unroll
    for (int k = 0; k < G; k++) {
        const int64_t g = g0 + min(k, ng - 1);  // a game past n repeats the last one; never written
        np[k] = min<u32>(plies[g], OTH_MOVES_STRIDE);
        row[k] = reinterpret_cast<const ulonglong2*>(pos) + (row_off ? row_off[g] : g * OTH_POS_STRIDE);
    }
    ulonglong2 term[G], b[G];
#pragma unroll
    for (int k = 0; k < G; k++) {
        term[k] = row[k][np[k]];
        b[k] = row[k][min(lane, np[k])];  // lanes past the game's positions reread its terminal row
    }
#pragma unroll
    for (int k = 0; k < G; k++) {
        if (k >= ng) break;
        const int vb = __popcll(term[k].x) - __popcll(term[k].y);  // value_for_black (41); white gets -vb (42)
        const int64_t jb = base[g0 + k];
        if (lane <= np[k]) td_update_pair<WORDS>(b[k], lane, np[k], vb, jb, lam_pow, keys, vals, words);
        for (u32 p = lane + 64; p <= np[k]; p += 64)  // games of more than 63 plies
            td_update_pair<WORDS>(row[k][p], p, np[k], vb, jb, lam_pow, keys, vals, words);
    }
}

// one thread per book record, in the learner's own order: row r is update
// pair 2r ('O') and 2r + 1 ('X'); its book's terminal record (book[0]) is row
// term_row[r] and l ** turn_left is lam_pow[lam_idx[r]]
__global__ __launch_bounds__(kBlock) void td_records_kernel(const u64* __restrict__ rows,
                                                            const int64_t* __restrict__ term_row,
                                                            const int32_t* __restrict__ lam_idx,
                                                            const double* __restrict__ lam_pow,
                                                            int64_t* __restrict__ keys, double* __restrict__ vals,
                                                            int64_t n) {
    const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (r >= n) return;
    const ulonglong2* rb = reinterpret_cast<const ulonglong2*>(rows);
    const ulonglong2 term = rb[term_row[r]];
    const int vb = __popcll(term.x) - __popcll(term.y);  // value_for_black (41); white gets -vb (42)
    const double lam = lam_pow[lam_idx[r]];
    const ulonglong2 b = rb[r];
    keys[2 * r] = td_key(b, OTH_BLACK);
    vals[2 * r] = (double)vb * lam;
    keys[2 * r + 1] = td_key(b, OTH_WHITE);
    vals[2 * r + 1] = (double)(-vb) * lam;
}

// one thread per key segment, strictly sequential in stream order (the EMA is
// order-dependent and bit-exact parity needs Python's rounding: no contraction).
// A key's updates number up to ~2 per game (the first plies), so long segments
// are software-pipelined: a ring of three chunks keeps 2 * kTdChunk loads in
// flight while the dependent multiply/add/select chain consumes the third
// (profiles/design_history_r01_r04.md §10: 69.5 ms for a 262,144-game batch).
constexpr int kTdChunk = 16;
__device__ __forceinline__ double td_step(double v, double x, double a, double oma) {
#pragma clang fp contract(off)
    return (v == 0.0) ? x : v * oma + x * a;
}
__device__ __forceinline__ void td_load(double (&b)[kTdChunk], const double* vals, int64_t i, int64_t last) {
#pragma unroll
    for (int k = 0; k < kTdChunk; k++) b[k] = vals[min(i + k, last)];  // clamped: always in bounds
}
__device__ __forceinline__ double td_run(double v, const double (&b)[kTdChunk], int m, double a, double oma) {
#pragma unroll
    for (int k = 0; k < kTdChunk; k++)
        if (k < m) v = td_step(v, b[k], a, oma);
    return v;
}
// a full chunk, speculating that no state in it is exactly 0 (the rule then
// reduces to v * oma + x * a, a two-op dependent chain with x * a off the
// chain); if any pre-update state was 0 the chunk is redone with the exact
// rule, so the result is identical either way
__device__ __forceinline__ double td_run_full(double v, const double (&b)[kTdChunk], double a, double oma) {
#pragma clang fp contract(off)
    double y[kTdChunk];
#pragma unroll
    for (int k = 0; k < kTdChunk; k++) y[k] = b[k] * a;
    // each step: the chain's multiply, a running min of |state| (exactly 0
    // iff some state was +-0; cheaper than a compare and an SGPR OR per
    // step), the chain's add -- one asm block, so the min issues in the
    // add's wait
    double w = v, mn = 1.0;
#pragma unroll
    for (int k = 0; k < kTdChunk; k++) {
        double t;
        asm("v_mul_f64 %[t], %[w], %[oma]\n\t"
            "v_min_f64 %[mn], %[mn], |%[w]|\n\t"
            "v_add_f64 %[w], %[t], %[y]"
            : [w] "+v"(w), [mn] "+v"(mn), [t] "=&v"(t)
            : [oma] "v"(oma), [y] "v"(y[k]));
    }
    return mn == 0.0 ? td_run(v, b, kTdChunk, a, oma) : w;
}
// the rule over vals[i, e) from state v, one thread: short ranges step by
// step; long ones software-pipelined (a ring of three chunks keeps 2 * kTdChunk
// loads in flight while the chain consumes the third)
__device__ __forceinline__ double td_range(double v, const double* __restrict__ vals, int64_t i, const int64_t e, double a,
                           double oma) {
    if (e - i < 3 * kTdChunk) {  // the common case: a handful of updates
        for (; i < e; i++) v = td_step(v, vals[i], a, oma);
        return v;
    }
    const int64_t last = e - 1;
    double b0[kTdChunk], b1[kTdChunk], b2[kTdChunk];
    td_load(b0, vals, i, last);
    td_load(b1, vals, i + kTdChunk, last);
    td_load(b2, vals, i + 2 * kTdChunk, last);
    for (; i + 3 * kTdChunk <= e; i += 3 * kTdChunk) {
        v = td_run_full(v, b0, a, oma);
        td_load(b0, vals, i + 3 * kTdChunk, last);
        v = td_run_full(v, b1, a, oma);
        td_load(b1, vals, i + 4 * kTdChunk, last);
        v = td_run_full(v, b2, a, oma);
        td_load(b2, vals, i + 5 * kTdChunk, last);
    }
    const int r = (int)(e - i);  // 0 .. 3*kTdChunk-1 left, already in b0, b1, b2
    v = td_run(v, b0, r, a, oma);
    v = td_run(v, b1, r - kTdChunk, a, oma);
    v = td_run(v, b2, r - 2 * kTdChunk, a, oma);
    return v;
}
// long_min: segments at least this long belong to td_ema_long_kernel (0: none).
// SHORT: every segment here is shorter than 3 chunks (long_min <= 3 * kTdChunk),
// so the kernel has no ring of loads and needs a fraction of the registers:
// more waves in flight for the millions of 1- to 3-update keys.
constexpr int kTdEmaPre = 8;
template <bool SHORT>
__global__ __launch_bounds__(kBlock) void td_ema_kernel(const double* __restrict__ vals,
                                                        const int64_t* __restrict__ seg_off,
                                                        const double* __restrict__ init, double a, double oma,
                                                        double* __restrict__ out, int64_t n_seg, int64_t long_min) {
    const int64_t s = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (s >= n_seg) return;
    int64_t i = seg_off[s];
    const int64_t e = seg_off[s + 1];
    if (long_min > 0 && e - i >= long_min) return;
    double v = init ? init[s] : 0.0;
    if (SHORT) {
        // the first kTdEmaPre values loaded together (predicated), so
        // most keys (1 to a few updates) wait on one round trip for them
        // rather than one per update; the rest one by one
        constexpr int kPre = kTdEmaPre;
        double x[kPre > 0 ? kPre : 1];
#pragma unroll
        for (int k = 0; k < kPre; k++) x[k] = i + k < e ? vals[i + k] : 0.0;
#pragma unroll
        for (int k = 0; k < kPre; k++)
            if (i + k < e) v = td_step(v, x[k], a, oma);
        for (i += kPre; i < e; i++) v = td_step(v, vals[i], a, oma);
        out[s] = v;
    } else {
        out[s] = td_range(v, vals, i, e, a, oma);
    }
}

// Speculative split of a very long segment (the opening position's key gets
// one update per game and side; the first plies' keys a fraction of that)
// into parts of kSpecLen updates, run side by side.  The rule is a
// contraction (|1 - a| < 1): two runs over the same values from different
// states approach each other by |1 - a| per step and, once a rounding maps
// them to the same double, mostly stay equal.  So the lane of part p > 0
// guesses the state at the start of its part by a warm-up run over the
// `warm` values before it, from state 0 (the rule then starts at the first
// value itself), or exactly, from the key's initial state, when the part
// starts within `warm` of the segment; `warm` is sized by the launcher so
// that |1 - a|^warm < 2^-64.  Lane p then runs its part from the guess.  A
// part whose guess equals the end state of the part before, itself exact, ran
// from the exact state; part 0 is exact.  The guesses that missed (the last
// ulp had not merged yet: ~1 in 1,000 parts, tools/diag/td_spec_probe.py) are
// rerun from the end state of the part before, and the check repeats until
// every part matches its predecessor; each pass fixes at least the first
// miss.  Every result is thus the sequential one; speculation only decides
// how fast it comes.
//
// Three launches: td_spec_plan_kernel lists the keys to split with their
// parts and work items (a wave's 64 consecutive parts); td_spec_parts_kernel
// runs every work item as a one-wave block, so one key's parts spread over
// as many CUs as it has work items; td_spec_fix_kernel checks each key's
// parts in order and reruns the misses.  (Round 4's first versions ran a
// key's parts in one block of 256 or 512 lanes: 0.8-2 us a round of 16 steps,
// growing with the lanes of the block -- one CU's load path -- 320-430 us per
// launch for the opening key.)
// Feeding a wave: each lane streams its own range, so lane-private loads would
// touch 64 cache lines per wave instruction.  Instead the wave moves its
// parts' values in rounds of kTdChunk per lane: it loads the round's 64 x 16
// doubles cooperatively (one load instruction covers 4 rows of 16 consecutive
// doubles) through a buffer descriptor that advances 16 doubles a round
// (fixed per-lane offsets, no address arithmetic; the descriptor's range check
// reads 0 past the key), parks them in LDS rows padded by one double (bank
// spread), and each lane then runs its 16 steps from its row.  Loads run
// kSpecAhead rounds ahead in registers; LDS is double-buffered.  Part lengths
// and warm-ups are whole rounds, so every lane's guess falls on a round
// boundary and only a key's last part ends inside a round.
constexpr int kSpecLanes = 64;          // parts per work item (one wave)
constexpr int kSpecLen = 1040;          // updates per part: 65 rounds, an odd number (rows
                                        // of one round an odd multiple of 128 B apart)
constexpr int kSpecRow = kTdChunk + 1;  // LDS doubles per part row (padded)
constexpr int kSpecAhead = 3;           // rounds of loads in flight (register sets)
constexpr int kSpecRowsPerLoad = kSpecLanes / kTdChunk;
struct SpecWave {
    double stage[2][kSpecLanes * kSpecRow];
    int start[kSpecLanes];  // a lane's stream start, relative to the key's first value
    int rounds;
};
struct SpecPlanEntry {
    int64_t s, part_base, item_base, n_parts;
};
constexpr int kSpecHdr = 8;  // int64 header of the scratch: [0] keys split, [1] work items, [2] parts, [3] counter
constexpr int64_t kSpecMaxLen = 1ll << 27;  // longer keys (beyond any batch in HBM) stay sequential
// keys of >= 3 warm-ups are split (at a = 0.03: 5,826 updates, the single-lane
// chain's longest as in round 3; at 4 warm-ups of the longer round-4 warm-up,
// 7,768, the long-key kernel took 199 us against 130)
constexpr int64_t kSpecMinWarms = 3;
__device__ __forceinline__ int64_t uniform64(int64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// the wave streams [ws, j) of the key's values kv[0, n) from state v (live
// lanes only; ws and j relative to kv), recording in g its state at i (a
// round boundary at or after ws).  kv and n wave-uniform.
__device__ __forceinline__ void spec_stream(const double* kv, int n, bool live, int ws, int i, int j, double& v,
                                            double& g, double a, double oma, SpecWave& sh) {
    const int p = threadIdx.x;
    const int rounds_p = live ? (j - ws + kTdChunk - 1) / kTdChunk : 0;
    const int chk = (i - ws) / kTdChunk;
    sh.start[p] = live ? ws : 0;
    int rmax = rounds_p;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) rmax = max(rmax, __shfl_xor(rmax, o));
    const int rounds = __builtin_amdgcn_readfirstlane(rmax);
    wave_sync();
    // this lane's load slots: row k * kSpecRowsPerLoad + p / 16, column p % 16
    int off[kTdChunk];
#pragma unroll
    for (int k = 0; k < kTdChunk; k++) off[k] = (sh.start[k * kSpecRowsPerLoad + (p >> 4)] + (p & 15)) * 8;
    auto fetch = [&](double(&r)[kTdChunk], int round) {
        const int base = round * kTdChunk;
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(kv + base), (short)0, max(n - base, 0) * 8,
                                                            0x00020000);
#pragma unroll
        for (int k = 0; k < kTdChunk; k++)
            r[k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off[k], 0, 0));
    };
    auto park = [&](const double(&r)[kTdChunk], int buf) {
#pragma unroll
        for (int k = 0; k < kTdChunk; k++)
            sh.stage[buf][(k * kSpecRowsPerLoad + (p >> 4)) * kSpecRow + (p & 15)] = r[k];
    };
    double rg[kSpecAhead][kTdChunk];
#pragma unroll
    for (int u = 0; u < kSpecAhead; u++) fetch(rg[u], u);
    for (int r0 = 0; r0 < rounds; r0 += kSpecAhead) {
#pragma unroll
        for (int u = 0; u < kSpecAhead; u++) {
            const int r = r0 + u;
            if (r >= rounds) break;  // wave-uniform
            park(rg[u], r & 1);
            fetch(rg[u], r + kSpecAhead);
            wave_sync();  // round r parked (a wave's LDS ops are in order)
            if (r < rounds_p) {
                if (r == chk) g = v;
                double x[kTdChunk];
                const double* row = &sh.stage[r & 1][p * kSpecRow];
#pragma unroll
                for (int k = 0; k < kTdChunk; k++) x[k] = row[k];
                const int m = j - ws - r * kTdChunk;
                v = m >= kTdChunk ? td_run_full(v, x, a, oma) : td_run(v, x, m, a, oma);
            }
        }
    }
    wave_sync();  // the stage and start rows are free for the next stream
}
// the parts of a key of n updates
__device__ __forceinline__ int64_t spec_parts(int64_t n) { return (n + kSpecLen - 1) / kSpecLen; }

// the keys of >= spec_min updates among the long keys, compacted into the
// plan (slot order is arbitrary: each key's result is its own) with their
// part counts; hdr[3] counts them (zeroed by the launcher)
__global__ __launch_bounds__(kBlock) void td_spec_select_kernel(const int64_t* __restrict__ seg_off,
                                                                const int64_t* __restrict__ long_idx, int64_t n_long,
                                                                int64_t spec_min, int64_t* __restrict__ hdr,
                                                                SpecPlanEntry* __restrict__ plan) {
    const int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n_long) return;
    const int64_t s = long_idx[k], n = seg_off[s + 1] - seg_off[s];
    if (n < spec_min || n > kSpecMaxLen) return;
    const int64_t slot = (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(hdr + 3), 1ull);
    plan[slot] = SpecPlanEntry{s, 0, 0, spec_parts(n)};
}
// one block: the running offsets of the selected keys' parts and work items
// (exclusive scans over the plan), and the totals into hdr[0..2].  cap: the
// parts the scratch holds (the caller's n_values sizes it).  A key whose parts
// would end past cap (n_values below seg_off[n_seg], a caller error the
// header names) gets no parts and no work items: td_spec_fix_kernel then runs
// it sequentially, so no part is ever written out of bounds.
// one block of kPlanThreads: beside the short keys' kernel (the EMA's side
// streams) a block of 1,024 threads waited 40-67 us for a CU with room for it
constexpr int kPlanThreads = 256, kPlanWaves = kPlanThreads / 64;
__global__ __launch_bounds__(kPlanThreads) void td_spec_plan_kernel(int64_t* __restrict__ hdr,
                                                                    SpecPlanEntry* __restrict__ plan, int64_t cap) {
    __shared__ u32 wsum[2][kPlanWaves];
    __shared__ int64_t carry[2];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t n_spec = hdr[3];
    if (t < 2) carry[t] = 0;
    __syncthreads();
    // an inclusive block scan of x (channel c): returns the exclusive prefix
    // over the keys before this one, the carry of earlier rounds included
    auto block_excl = [&](u32 x, int c) -> int64_t {
        const u32 incl = wave_incl_scan(x);
        if (lane == 63) wsum[c][wv] = incl;
        __syncthreads();
        u32 before = 0;
        for (int w2 = 0; w2 < wv; w2++) before += wsum[c][w2];
        return carry[c] + before + incl - x;
    };
    for (int64_t t0 = 0; t0 < n_spec; t0 += kPlanThreads) {
        const int64_t k = t0 + t;
        u32 P = k < n_spec ? (u32)plan[k].n_parts : 0u;
        const int64_t pbase = block_excl(P, 0);
        if (pbase + P > cap) P = 0;  // does not fit: sequential in td_spec_fix_kernel
        const u32 C = (P + kSpecLanes - 1) / kSpecLanes;
        const int64_t ibase = block_excl(C, 1);
        if (k < n_spec) {
            plan[k].n_parts = P;
            plan[k].part_base = pbase;
            plan[k].item_base = ibase;
        }
        __syncthreads();
        if (t < 2) {
            u32 tot = 0;
            for (int w2 = 0; w2 < kPlanWaves; w2++) tot += wsum[t][w2];
            carry[t] += tot;
        }
        __syncthreads();
    }
    if (t == 0) {
        hdr[0] = n_spec;
        hdr[1] = carry[1];
        hdr[2] = carry[0];
    }
}
// the key of work item w: the last plan entry whose first item is <= w
__device__ __forceinline__ int64_t spec_key_of(const SpecPlanEntry* plan, int64_t n_spec, int64_t w) {
    int64_t lo = 0, hi = n_spec - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (plan[mid].item_base <= w) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
// one wave per work item: parts q = 64 c + lane of its key, guesses and end states out
// the parts of block `blk` of `grid` (a grid-stride loop over the work items)
__device__ __forceinline__ void td_spec_parts_body(int64_t blk, int64_t grid, const double* __restrict__ vals,
                                                   const int64_t* __restrict__ seg_off,
                                                   const double* __restrict__ init, double a, double oma,
                                                   const int64_t* __restrict__ hdr,
                                                   const SpecPlanEntry* __restrict__ plan, double* __restrict__ guess,
                                                   double* __restrict__ fin, int warm16, SpecWave& sh) {
    const int64_t n_spec = uniform64(hdr[0]), items = uniform64(hdr[1]);
    for (int64_t w = blk; w < items; w += grid) {
        const int64_t key = uniform64(spec_key_of(plan, n_spec, w));
        const int64_t s = uniform64(plan[key].s), pb = uniform64(plan[key].part_base);
        const int64_t ib = uniform64(plan[key].item_base), np = uniform64(plan[key].n_parts);
        const int64_t b = uniform64(seg_off[s]);
        const int n = (int)uniform64(seg_off[s + 1] - b);
        const int64_t q = (w - ib) * kSpecLanes + threadIdx.x;
        const bool live = q < np;
        const int i = (int)q * kSpecLen, j = live ? min(i + kSpecLen, n) : i, ws = max(0, i - warm16);
        double v = (ws == 0 && init) ? init[s] : 0.0, g = v;
        spec_stream(vals + b, n, live, ws, i, j, v, g, a, oma, sh);
        if (live) {
            guess[pb + q] = g;
            fin[pb + q] = v;
        }
    }
}
__global__ __launch_bounds__(kSpecLanes) void td_spec_parts_kernel(const double* __restrict__ vals,
                                                                   const int64_t* __restrict__ seg_off,
                                                                   const double* __restrict__ init, double a,
                                                                   double oma, const int64_t* __restrict__ hdr,
                                                                   const SpecPlanEntry* __restrict__ plan,
                                                                   double* __restrict__ guess,
                                                                   double* __restrict__ fin, int warm16) {
    __shared__ SpecWave sh;
    td_spec_parts_body(blockIdx.x, gridDim.x, vals, seg_off, init, a, oma, hdr, plan, guess, fin, warm16, sh);
}
// one wave per split key: its parts checked in order, 64 at a time; missed
// guesses rerun from their predecessor's end state until all match
__global__ __launch_bounds__(kSpecLanes) void td_spec_fix_kernel(const double* __restrict__ vals,
                                                                 const int64_t* __restrict__ seg_off,
                                                                 const double* __restrict__ init, double a,
                                                                 double oma, const int64_t* __restrict__ hdr,
                                                                 const SpecPlanEntry* __restrict__ plan,
                                                                 const double* __restrict__ guess,
                                                                 const double* __restrict__ fin,
                                                                 double* __restrict__ out) {
    __shared__ SpecWave sh;
    const int lane = threadIdx.x;
    const int64_t n_spec = uniform64(hdr[0]);
    for (int64_t key = blockIdx.x; key < n_spec; key += gridDim.x) {
        const int64_t s = uniform64(plan[key].s), pb = uniform64(plan[key].part_base);
        const int64_t np = uniform64(plan[key].n_parts);
        const int64_t b = uniform64(seg_off[s]);
        const int n = (int)uniform64(seg_off[s + 1] - b);
        if (np == 0) {  // parts past the scratch (td_spec_plan_kernel): the whole key on lane 0
            double v = init ? init[s] : 0.0, unused = v;
            spec_stream(vals + b, n, lane == 0, 0, 0, n, v, unused, a, oma, sh);
            if (lane == 0) out[s] = v;
            continue;
        }
        double prev = 0.0;  // the end state of the part before this chunk's first
        for (int64_t c0 = 0; c0 < np; c0 += kSpecLanes) {
            const int64_t q = c0 + lane;
            const bool live = q < np;
            double g = live ? guess[pb + q] : 0.0, f = live ? fin[pb + q] : 0.0;
            for (int pass = 0; pass <= kSpecLanes; pass++) {  // each pass fixes the first miss at least
                double pred = __shfl_up(f, 1);
                if (lane == 0) pred = prev;
                const bool miss = live && q > 0 && __double_as_longlong(g) != __double_as_longlong(pred);
                if (!__ballot(miss)) break;  // wave-uniform
                const int i = (int)q * kSpecLen, j = miss ? min(i + kSpecLen, n) : i;
                double w = pred, unused = pred;
                spec_stream(vals + b, n, miss, i, i, j, w, unused, a, oma, sh);
                if (miss) {
                    g = pred;
                    f = w;
                }
            }
            prev = __shfl(f, (int)min<int64_t>(kSpecLanes - 1, np - 1 - c0));
        }
        if (lane == 0) out[s] = prev;
    }
}
// the scratch of the split: header, plan entries, guesses and end states
inline size_t spec_scratch_bytes(int64_t n_long, int64_t n_values) {
    const int64_t parts = n_values / kSpecLen + n_long + 1;  // sum of ceil(n / kSpecLen) over <= n_long keys
    return sizeof(int64_t) * kSpecHdr + sizeof(SpecPlanEntry) * (size_t)std::max<int64_t>(n_long, 1) +
           2 * sizeof(double) * (size_t)parts;
}

// One long segment per single-wave block.  A thread alone is bound by how many
// loads it keeps in flight (~30 dwordx2: the 524,288-update opening key of a
// 262,144-game batch took ~13 ms); here the whole wave stages the segment
// through LDS with coalesced loads, double-buffered, and lane 0 runs the chain
// from LDS while the next stage is in flight, so the time is the chain's.
// (round 5: 1,024 before; at 33 KiB of LDS per one-wave block only 4 keys'
// chains ran per CU: 131 -> 92 us per batch at 512, 106-110 at 256)
constexpr int kTdStage = 512;         // doubles per LDS stage
constexpr int kTdStageLoads = kTdStage / 64;   // loads per lane per stage
// (ystage rows padded by one chunk: the chain prefetches the next chunk's y
// unconditionally)
struct LongStage {
    double stage[2][kTdStage], ystage[2][kTdStage + kTdChunk];
};
__device__ __forceinline__ void td_ema_long_body(int64_t blk, const double* __restrict__ vals,
                                                 const int64_t* __restrict__ seg_off,
                                                 const double* __restrict__ init, double a, double oma,
                                                 double* __restrict__ out, const int64_t* __restrict__ long_idx,
                                                 int64_t warm, LongStage& ls) {
    double(&stage)[2][kTdStage] = ls.stage;
    double(&ystage)[2][kTdStage + kTdChunk] = ls.ystage;
    const int lane = threadIdx.x;
    const int64_t s = long_idx[blk];
    const int64_t b = seg_off[s], e = seg_off[s + 1];
    if (warm > 0 && e - b >= kSpecMinWarms * warm && e - b <= kSpecMaxLen) return;  // a split key (td_spec_*)
    const int64_t n_stage = (e - b + kTdStage - 1) / kTdStage;
    double r[kTdStageLoads];
    auto fetch = [&](int64_t c) {
#pragma unroll
        for (int k = 0; k < kTdStageLoads; k++) {
            const int64_t idx = b + c * kTdStage + k * 64 + lane;
            r[k] = idx < e ? vals[idx] : 0.0;
        }
    };
    auto park = [&](int buf) {
#pragma clang fp contract(off)
#pragma unroll
        for (int k = 0; k < kTdStageLoads; k++) {
            stage[buf][k * 64 + lane] = r[k];
            ystage[buf][k * 64 + lane] = r[k] * a;  // the chain's x * a, off its critical path
        }
    };
    fetch(0);
    park(0);
    __syncthreads();
    double v = (lane == 0 && init) ? init[s] : 0.0;
    for (int64_t c = 0; c < n_stage; c++) {
        if (c + 1 < n_stage) fetch(c + 1);  // in flight while lane 0 runs stage c
        if (lane == 0) {
            // the chain; y = x * a was computed by the staging lanes
            const double* x = stage[c & 1];
            const double* y = ystage[c & 1];
            const int m = (int)min<int64_t>(kTdStage, e - b - c * kTdStage);
            // One lane issues this chain alone, so every instruction on it
            // costs its full issue time.  A chunk of kTdChunk steps runs the
            // two-op rule speculatively and tests its states for an exact 0
            // by one v_min_f64 of |state| per step (0 iff a state was +-0:
            // exact, no rounding; a compare per step doubled the chain's
            // time), then redoes the chunk with the exact rule if one was.
            // Each step is one asm block so that the min issues between the
            // chain's multiply and add, in the add's wait.
            auto chunk = [&](const double(&yk)[kTdChunk], int j0) {
                double w = v, mn = 1.0;
#pragma unroll
                for (int k = 0; k < kTdChunk; k++) {
                    double t;
                    asm("v_mul_f64 %[t], %[w], %[oma]\n\t"
                        "v_min_f64 %[mn], %[mn], |%[w]|\n\t"
                        "v_add_f64 %[w], %[t], %[y]"
                        : [w] "+v"(w), [mn] "+v"(mn), [t] "=&v"(t)
                        : [oma] "v"(oma), [y] "v"(yk[k]));
                }
                if (mn == 0.0) {  // a state was exactly 0: redo the chunk with the exact rule
                    double bk[kTdChunk];
#pragma unroll
                    for (int k = 0; k < kTdChunk; k++) bk[k] = x[j0 + k];
                    w = td_run(v, bk, kTdChunk, a, oma);
                }
                v = w;
            };
            // two chunk buffers: the next chunk's y is read from LDS while a
            // chunk runs (reads past m stay in the padded row, unused)
            double ya[kTdChunk], yb[kTdChunk];
            auto load = [&](double(&yk)[kTdChunk], int j0) {
#pragma unroll
                for (int k = 0; k < kTdChunk; k++) yk[k] = y[j0 + k];
            };
            int j = 0;
            load(ya, 0);
            for (; j + 2 * kTdChunk <= m; j += 2 * kTdChunk) {
                load(yb, j + kTdChunk);
                chunk(ya, j);
                load(ya, j + 2 * kTdChunk);
                chunk(yb, j + kTdChunk);
            }
            if (j + kTdChunk <= m) {
                chunk(ya, j);
                j += kTdChunk;
            }
            double bk[kTdChunk];
#pragma unroll
            for (int k = 0; k < kTdChunk; k++) bk[k] = x[min(j + k, kTdStage - 1)];
            v = td_run(v, bk, m - j, a, oma);
        }
        if (c + 1 < n_stage) park((c + 1) & 1);
        __syncthreads();
    }
    if (lane == 0) out[s] = v;
}
__global__ __launch_bounds__(64) void td_ema_long_kernel(const double* __restrict__ vals,
                                                         const int64_t* __restrict__ seg_off,
                                                         const double* __restrict__ init, double a, double oma,
                                                         double* __restrict__ out,
                                                         const int64_t* __restrict__ long_idx, int64_t warm) {
    __shared__ LongStage ls;
    td_ema_long_body(blockIdx.x, vals, seg_off, init, a, oma, out, long_idx, warm, ls);
}
// The long keys and the split keys' parts in one launch (late round 5): blocks
// [0, parts_grid) run the parts (a grid-stride loop over the work items), the
// rest the long keys; the parts first, so that their few long-running blocks
// are dispatched at once rather than behind thousands of long keys.  Both are latency-bound chains on
// few waves; launched one after the other they ran ~90 + ~95 us, side by side
// about as long as the longer.  One LDS area serves either role.
union LongOrParts {
    LongStage ls;
    SpecWave sw;
};
__global__ __launch_bounds__(64) void td_ema_long_parts_kernel(const double* __restrict__ vals,
                                                               const int64_t* __restrict__ seg_off,
                                                               const double* __restrict__ init, double a, double oma,
                                                               double* __restrict__ out,
                                                               const int64_t* __restrict__ long_idx, int64_t warm,
                                                               int64_t n_long, const int64_t* __restrict__ hdr,
                                                               const SpecPlanEntry* __restrict__ plan,
                                                               double* __restrict__ guess, double* __restrict__ fin,
                                                               int warm16, int64_t parts_grid) {
    __shared__ LongOrParts lp;
    const int64_t blk = blockIdx.x;
    if (blk < parts_grid)
        td_spec_parts_body(blk, parts_grid, vals, seg_off, init, a, oma, hdr, plan, guess, fin, warm16, lp.sw);
    else
        td_ema_long_body(blk - parts_grid, vals, seg_off, init, a, oma, out, long_idx, warm, lp.ls);
}

inline int status(hipError_t e) { return e == hipSuccess ? OTH_OK : -(int)e; }

// launch geometry of the rollout kernel, resolved once per process (device 0 of
// the calling thread's current device).  Env overrides are tuning knobs for
// tools/diag only: OTH_ROLLOUT_BLOCKS_PER_CU.
struct Tuning {
    unsigned resident_blocks[3];  // per policy
    unsigned random_big_blocks;   // the random policy at >= kBigLaunch games
};

int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) : dflt;
}

// per-device launch geometry (a process may drive several GPUs), resolved on
// first use; the only state the library keeps, and none of it on the device
constexpr int kMaxDevices = 64;
constexpr int kMaxBlocksPerCu = 5;
constexpr int kRandomBlocksPerCu = 3;
constexpr int64_t kBigLaunch = 1 << 22;  // games: a launch this large amortises its own tail
struct DeviceState {
    std::atomic<int> ready{0};
    Tuning tuning;
};
DeviceState g_dev[kMaxDevices];
std::mutex g_dev_mu;

DeviceState* device_state() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDevices) return nullptr;
    DeviceState& d = g_dev[dev];
    if (d.ready.load(std::memory_order_acquire)) return &d;
    std::lock_guard<std::mutex> lock(g_dev_mu);
    if (!d.ready.load(std::memory_order_relaxed)) {
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const void* kern[3] = {reinterpret_cast<const void*>(rollout_kernel<OTH_POLICY_RANDOM, false>),
                               reinterpret_cast<const void*>(rollout_kernel<OTH_POLICY_GREEDY, false>),
                               reinterpret_cast<const void*>(rollout_kernel<OTH_POLICY_EVAL, false>)};
        for (int p = 0; p < 3; p++) {
            int per_cu = 0;
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern[p], kBlock, 0);
            // the random policy: 3 blocks of 4 waves per CU, so that two launches
            // in flight (2 streams, as INTEGRATION.md advises) are resident side
            // by side (6 of the 7 waves/SIMD its 70 VGPRs allow): 1.97e11
            // env-steps/s against 1.92e11 at 5 and 1.94e11 at 4 (tools/diag/bpc_k.sh,
            // 1M games per launch, 100 timed steps; 1.85-1.89e11 against
            // 1.83-1.84e11 at 20).  A launch of >= kBigLaunch games keeps 5: it
            // runs alone for most of its life (16M games, one stream: 2.0e11 at 5,
            // 1.91e11 at 3).  The 1-ply policies keep <= 5 (tools/diag/sweep_rollout.sh:
            // more waves only add batch-tail idle lanes)
            const int occ = per_cu;
            const int cap = p == OTH_POLICY_RANDOM ? kRandomBlocksPerCu : kMaxBlocksPerCu;
            per_cu = occ > 0 ? std::min(occ, cap) : 2;
            per_cu = env_int("OTH_ROLLOUT_BLOCKS_PER_CU", per_cu);
            d.tuning.resident_blocks[p] = (unsigned)(cus * per_cu);
            if (p == OTH_POLICY_RANDOM) {
                const int big = env_int("OTH_ROLLOUT_BLOCKS_PER_CU", occ > 0 ? std::min(occ, kMaxBlocksPerCu) : 2);
                d.tuning.random_big_blocks = (unsigned)(cus * big);
            }
        }
        d.ready.store(1, std::memory_order_release);
    }
    return &d;
}
inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }
inline int launched() { return status(hipGetLastError()); }
// the TD update stream (td_updates_wave_kernel)
static int td_updates_launch(const u64* pos, const int64_t* row_off, const uint8_t* plies, const int64_t* base,
                             const double* lam_pow, int64_t* keys, double* vals, u64* words, int64_t n, hipStream_t s) {
    (words ? td_updates_wave_kernel<true> : td_updates_wave_kernel<false>)<<<
        blocks_for((n + kTdUpdGames - 1) / kTdUpdGames * 64), kBlock, 0, s>>>(pos, row_off, plies, base, lam_pow, keys,
                                                                               vals, words, n);
    return launched();
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

const char* oth_version(void) { return OTH_VERSION; }

int oth_reset(uint64_t* boards, uint8_t* turn, uint8_t* nturn, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && !boards)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    reset_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(boards, turn, nturn, n);
    return launched();
}

int oth_legal(const uint64_t* boards, const uint8_t* turn, uint64_t* legal, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!boards || !turn || !legal))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    legal_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(boards, turn, legal, n);
    return launched();
}

int oth_step(const uint64_t* boards_in, const uint8_t* turn_in, const uint8_t* move, uint64_t* boards_out,
             uint8_t* turn_out, uint64_t* flips, uint64_t* legal_next, int8_t* ret, uint8_t* nturn, int64_t n,
             void* stream) {
    if (n < 0 || (n > 0 && (!boards_in || !turn_in || !move))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    step_kernel<<<blocks_for((n + kStepPerThread - 1) / kStepPerThread), kBlock, 0, (hipStream_t)stream>>>(
        boards_in, turn_in, move, boards_out, turn_out, flips, legal_next, ret, nturn, n);
    return launched();
}

int oth_hands(const uint64_t* own, const uint64_t* hostile, const int64_t* x, const int64_t* y, const int64_t* dx,
              const int64_t* dy, uint8_t* count, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!own || !hostile || !x || !y || !dx || !dy || !count))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    hands_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(own, hostile, x, y, dx, dy, count, n);
    return launched();
}

int oth_result(const uint64_t* boards, uint8_t* n_black, uint8_t* n_white, int8_t* diff, uint8_t* terminal,
               int64_t n, void* stream) {
    if (n < 0 || (n > 0 && !boards)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    result_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(boards, n_black, n_white, diff, terminal, n);
    return launched();
}

namespace {
struct RunnerSpec {
    int n_rand_a, n_rand_b, swap;
    uint8_t* a_black;
};
int rollout_launch(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                   int n_random, const int8_t* w_black, const int8_t* w_white, uint64_t* final_boards, int8_t* diff,
                   uint8_t* plies, uint8_t* moves, int64_t* hist, uint64_t* work, int64_t n, void* stream,
                   const RunnerSpec* run = nullptr) {
    RolloutArgs a;
    a.n_rand_a = run ? (u32)std::min(run->n_rand_a, 10) : 0u;  // N_RAND_HAND_UNTIL (game_runner.py:6, 117-118)
    a.n_rand_b = run ? (u32)std::min(run->n_rand_b, 10) : 0u;
    a.swap = run ? run->swap : 0;
    a.a_black = run ? run->a_black : nullptr;
    a.start = start;
    a.start_turn = start_turn;
    a.seed_state = mix64(seed + GOLDEN64);
    a.game_id0 = game_id0;
    a.n_random = n_random;
    a.final_boards = final_boards;
    a.diff = diff;
    a.plies = plies;
    a.moves = moves;
    a.hist = (long long*)hist;
    a.n = n;
    for (int k = 0; k < OTH_EVAL_WEIGHTS; k++) {
        a.ew[0].w[k] = w_black ? w_black[k] : 0;
        a.ew[1].w[k] = w_white ? w_white[k] : 0;
    }
    DeviceState* ds = device_state();
    if (!ds) return status(hipErrorInvalidDevice);
    const Tuning& t = ds->tuning;
    const int64_t max_blocks = (n + kBlock - 1) / kBlock;
    const unsigned resident =
        policy == OTH_POLICY_RANDOM && n >= kBigLaunch ? t.random_big_blocks : t.resident_blocks[policy];
    const unsigned grid = (unsigned)std::min<int64_t>(max_blocks, (int64_t)resident);
    a.work = reinterpret_cast<unsigned long long*>(work);
    // OTH_COOP_CAP=0 (tests only): every 1-ply choice by its own lane
    // (lane_choose), so the per-lane path runs from ordinary positions
    a.coop_cap = env_int("OTH_COOP_CAP", 1) == 0 ? 0u : 1u;
    a.last_ticket = 64ull * ((u64)((n + 63) / 64) + (u64)grid * (kBlock / 64) - 1ull);
    // (game indices are parked as 32 bits)
    a.handoff_k = n <= 0xFFFFFFFFll
                      ? (u32)std::min(std::max(env_int("OTH_HANDOFF_K", (int)kHandoffK), 0), (int)kHandoffKMax)
                      : 0u;
    hipStream_t st = (hipStream_t)stream;
    if (run) {
        if (policy == OTH_POLICY_EVAL) {
            if (moves) rollout_kernel<OTH_POLICY_EVAL, true, true><<<grid, kBlock, 0, st>>>(a);
            else rollout_kernel<OTH_POLICY_EVAL, false, true><<<grid, kBlock, 0, st>>>(a);
        } else {
            if (moves) rollout_kernel<OTH_POLICY_GREEDY, true, true><<<grid, kBlock, 0, st>>>(a);
            else rollout_kernel<OTH_POLICY_GREEDY, false, true><<<grid, kBlock, 0, st>>>(a);
        }
    } else if (policy == OTH_POLICY_EVAL) {
        if (moves) rollout_kernel<OTH_POLICY_EVAL, true><<<grid, kBlock, 0, st>>>(a);
        else rollout_kernel<OTH_POLICY_EVAL, false><<<grid, kBlock, 0, st>>>(a);
    } else if (policy == OTH_POLICY_GREEDY) {
        if (moves) rollout_kernel<OTH_POLICY_GREEDY, true><<<grid, kBlock, 0, st>>>(a);
        else rollout_kernel<OTH_POLICY_GREEDY, false><<<grid, kBlock, 0, st>>>(a);
    } else {
        if (moves)
            rollout_kernel<OTH_POLICY_RANDOM, true><<<grid, kBlock, rec_stage_bytes(OTH_POLICY_RANDOM, true), st>>>(a);
        else rollout_kernel<OTH_POLICY_RANDOM, false><<<grid, kBlock, 0, st>>>(a);
    }
    return launched();
}
}  // namespace

int oth_rollout(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                int n_random, uint64_t* final_boards, int8_t* diff, uint8_t* plies, uint8_t* moves, int64_t* hist,
                uint64_t* work, int64_t n, void* stream) {
    if (n < 0 || !work || (policy != OTH_POLICY_RANDOM && policy != OTH_POLICY_GREEDY)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return rollout_launch(start, start_turn, seed, game_id0, policy, n_random, nullptr, nullptr, final_boards, diff,
                          plies, moves, hist, work, n, stream);
}

int oth_rollout_eval(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                     int n_random, const int8_t* weights, uint64_t* final_boards, int8_t* diff, uint8_t* plies,
                     uint8_t* moves, int64_t* hist, uint64_t* work, int64_t n, void* stream) {
    if (n < 0 || !weights || !work) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return rollout_launch(start, start_turn, seed, game_id0, OTH_POLICY_EVAL, n_random, weights, weights, final_boards,
                          diff, plies, moves, hist, work, n, stream);
}

int oth_rollout_match(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0,
                      int n_random, const int8_t* weights_black, const int8_t* weights_white, uint64_t* final_boards,
                      int8_t* diff, uint8_t* plies, uint8_t* moves, int64_t* hist, uint64_t* work, int64_t n,
                      void* stream) {
    if (n < 0 || !weights_black || !weights_white || !work) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return rollout_launch(start, start_turn, seed, game_id0, OTH_POLICY_EVAL, n_random, weights_black, weights_white,
                          final_boards, diff, plies, moves, hist, work, n, stream);
}

int oth_rollout_runner(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                       const int8_t* weights_a, const int8_t* weights_b, int n_rand_a, int n_rand_b, int swap_colours,
                       uint8_t* a_black, uint64_t* final_boards, int8_t* diff, uint8_t* plies, uint8_t* moves,
                       int64_t* hist, uint64_t* work, int64_t n, void* stream) {
    if (n < 0 || !work || (policy != OTH_POLICY_GREEDY && policy != OTH_POLICY_EVAL) ||
        (policy == OTH_POLICY_EVAL && (!weights_a || !weights_b)) || n_rand_a < 0 || n_rand_b < 0)
        return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    const RunnerSpec run{n_rand_a, n_rand_b, swap_colours != 0, a_black};
    return rollout_launch(start, start_turn, seed, game_id0, policy, 0, weights_a, weights_b, final_boards, diff,
                          plies, moves, hist, work, n, stream, &run);
}

int oth_replay(const uint64_t* start, const uint8_t* start_turn, const uint8_t* moves, const uint8_t* plies,
               uint64_t* pos_boards, uint8_t* pos_turn, uint8_t* pos_end, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!moves || !plies || !pos_boards))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    const bool staged = pos_turn || pos_end;
    const int vec_moves = ((uintptr_t)moves & 15) == 0;
    const int vec_out = (((uintptr_t)pos_turn | (uintptr_t)pos_end) & 15) == 0;
    replay_kernel<false><<<blocks_for(n), kBlock, staged ? kReplayStage : 0, (hipStream_t)stream>>>(
        start, start_turn, moves, plies, nullptr, pos_boards, pos_turn, pos_end, n, vec_moves, vec_out);
    return launched();
}

int oth_replay_rows(const uint64_t* start, const uint8_t* start_turn, const uint8_t* moves, const uint8_t* plies,
                    const int64_t* row_off, uint64_t* pos_boards, uint8_t* pos_turn, uint8_t* pos_end, int64_t n,
                    void* stream) {
    if (n < 0 || (n > 0 && (!moves || !plies || !row_off || !pos_boards))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    const bool staged = pos_turn || pos_end;
    const int vec_moves = ((uintptr_t)moves & 15) == 0;
    const int vec_out = (((uintptr_t)pos_turn | (uintptr_t)pos_end) & 15) == 0;
    replay_kernel<true><<<blocks_for(n), kBlock, staged ? kReplayStagePacked : 0, (hipStream_t)stream>>>(
        start, start_turn, moves, plies, row_off, pos_boards, pos_turn, pos_end, n, vec_moves, vec_out);
    return launched();
}


int oth_book_text(const uint64_t* boards, const uint8_t* turn, int64_t n, char* out, void* stream) {
    if (n < 0 || (n > 0 && (!boards || !turn || !out))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    book_text_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(boards, turn, n,
                                                                       reinterpret_cast<uint8_t*>(out),
                                                                       ((uintptr_t)out & 15) == 0);
    return launched();
}

int oth_book_parse(const char* text, int64_t stride, uint64_t* boards, uint8_t* turn, int64_t n, void* stream) {
    if (n < 0 || stride < 64 || (turn && stride < 66) || (n > 0 && (!text || !boards))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    const int vec = ((uintptr_t)text & 15) == 0 && stride % 16 == 0;
    book_parse_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(reinterpret_cast<const uint8_t*>(text),
                                                                        stride, boards, turn, n, vec);
    return launched();
}

int oth_features(const uint64_t* boards, const uint8_t* side, uint8_t* out, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!boards || !side || !out))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    features_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(boards, side, out, n);
    return launched();
}

int oth_eval(const uint64_t* boards, const uint8_t* side, const int8_t* weights, int32_t* out, int64_t n,
             void* stream) {
    if (n < 0 || !weights || (n > 0 && (!boards || !side || !out))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    EvalWeights ew;
    for (int k = 0; k < OTH_EVAL_WEIGHTS; k++) ew.w[k] = weights[k];
    eval_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(boards, side, ew, out, n);
    return launched();
}

int oth_td_updates(const uint64_t* pos_boards, const uint8_t* plies, const int64_t* base, const double* lam_pow,
                   int64_t* keys, double* values, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!pos_boards || !plies || !base || !lam_pow || !keys || !values))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return td_updates_launch(pos_boards, nullptr, plies, base, lam_pow, keys, values, nullptr, n, (hipStream_t)stream);
}

int oth_td_updates_packed(const uint64_t* pos_boards, const int64_t* row_off, const uint8_t* plies,
                          const int64_t* base, uint64_t* words, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!pos_boards || !plies || !base || !words))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return td_updates_launch(pos_boards, row_off, plies, base, nullptr, nullptr, nullptr, reinterpret_cast<u64*>(words),
                             n, (hipStream_t)stream);
}
int oth_td_updates_rows(const uint64_t* pos_boards, const int64_t* row_off, const uint8_t* plies, const int64_t* base,
                        const double* lam_pow, int64_t* keys, double* values, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!pos_boards || !row_off || !plies || !base || !lam_pow || !keys || !values)))
        return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    return td_updates_launch(pos_boards, row_off, plies, base, lam_pow, keys, values, nullptr, n, (hipStream_t)stream);
}

int oth_td_updates_records(const uint64_t* rows, const int64_t* term_row, const int32_t* lam_idx,
                           const double* lam_pow, int64_t* keys, double* values, int64_t n_rows, void* stream) {
    if (n_rows < 0 || (n_rows > 0 && (!rows || !term_row || !lam_idx || !lam_pow || !keys || !values)))
        return OTH_EINVAL;
    if (n_rows == 0) return OTH_OK;
    td_records_kernel<<<blocks_for(n_rows), kBlock, 0, (hipStream_t)stream>>>(rows, term_row, lam_idx, lam_pow, keys,
                                                                              values, n_rows);
    return launched();
}

int oth_td_ema(const double* values, const int64_t* seg_off, const double* init, double a, double one_minus_a,
               double* out, int64_t n_seg, void* stream) {
    if (n_seg < 0 || (n_seg > 0 && (!values || !seg_off || !out))) return OTH_EINVAL;
    if (n_seg == 0) return OTH_OK;
    td_ema_kernel<false><<<blocks_for(n_seg), kBlock, 0, (hipStream_t)stream>>>(values, seg_off, init, a,
                                                                                one_minus_a, out, n_seg, 0);
    return launched();
}

// Fork / join of the TD EMA's side streams (round 5).  The long keys' waves
// and the split keys' chain are latency-bound (a few thousand dependent
// chains) and ran after the short keys' kernel on the caller's stream; on two
// non-blocking side streams of the device they run beside it.  The side
// streams wait on an event recorded on the caller's stream at the fork, and
// the caller's stream waits on one event per side stream at the join, so
// everything after the call (on the caller's stream) sees all three kernels'
// outputs, as a single-stream call would.  A per-device mutex holds the fork
// to the join (the events are the device's, shared by every caller).
// Off by default, on with OTH_TD_EMA_FORK=1 in the environment: alone in a
// process it took 60-100 us off a 262,144-game batch (2.43 -> 2.33 ms,
// tools/diag/td_bench_ab.py), but inside bench.py, after the rollout lines
// have created their own streams, the same batch ran 2.41 -> 2.64 ms with it
// (the device's few hardware queues are then shared among more streams;
// profiles/r05_notes.md).
struct TdSides {
    std::mutex mu;
    bool made = false;
    int rc = OTH_OK;
    hipStream_t side[2] = {nullptr, nullptr};
    hipEvent_t fork = nullptr, join[2] = {nullptr, nullptr};
};
TdSides g_td_sides[kMaxDevices];
struct TdFork {
    TdSides* d = nullptr;
    hipStream_t s;
    int n = 0, rc = OTH_OK;
    std::unique_lock<std::mutex> lock;
    TdFork(hipStream_t caller, int n_sides) : s(caller) {
        static const int enabled = env_int("OTH_TD_EMA_FORK", 0);
        int dev = 0;
        if (n_sides <= 0 || !enabled || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return;
        d = &g_td_sides[dev];
        lock = std::unique_lock<std::mutex>(d->mu);
        if (!d->made) {
            d->made = true;
            // the side streams at the device's highest priority: their chains
            // are the EMA's critical path, so their waves take CU slots first
            int least = 0, greatest = 0;
            hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
            if (!env_int("OTH_TD_EMA_PRIO", 1)) greatest = least;
            for (int k = 0; k < 2 && e == hipSuccess; k++) {
                e = hipStreamCreateWithPriority(&d->side[k], hipStreamNonBlocking, greatest);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&d->join[k], hipEventDisableTiming);
            }
            if (e == hipSuccess) e = hipEventCreateWithFlags(&d->fork, hipEventDisableTiming);
            d->rc = status(e);
        }
        if ((rc = d->rc) != OTH_OK) return;
        rc = status(hipEventRecord(d->fork, s));
        for (int k = 0; k < n_sides && rc == OTH_OK; k++) {
            rc = status(hipStreamWaitEvent(d->side[k], d->fork, 0));
            if (rc == OTH_OK) n = k + 1;
        }
    }
    hipStream_t side(int k) const { return n > k ? d->side[k] : s; }
    // the caller's stream waits for the side streams; the first error wins
    int join(int rc0) {
        for (int k = 0; k < n; k++) {
            const int r = status(hipEventRecord(d->join[k], d->side[k]));
            const int w = r == OTH_OK ? status(hipStreamWaitEvent(s, d->join[k], 0)) : r;
            if (rc0 == OTH_OK) rc0 = w;
        }
        n = 0;
        return rc0;
    }
    ~TdFork() { join(OTH_OK); }
};

// warm-up length of the split's guesses for the rule's contraction |1 - a|:
// 4/3 of the smallest w with |1 - a|^w < 2^-64 (at w itself the two runs are
// still one ulp apart now and then: 4 misses among the first 40 split keys of
// a 262,144-game batch at a = 0.03; none at 4/3 w, and the reruns cost more
// than the longer warm-ups: tools/diag/td_spec_probe.py); 0 (no speculation)
// when the rule does not contract or w would pass 2^20.  OTH_TD_SPEC_WARM
// overrides it (tools/tests only: a tiny warm-up makes the guesses miss,
// which exercises the rerun passes).
static int64_t td_spec_warm(double oma) {
    if (const char* env = getenv("OTH_TD_SPEC_WARM")) return atoll(env);
    const double c = fabs(oma);
    if (!(c < 1.0)) return 0;
    if (c == 0.0) return 1;
    const double w = ceil(-64.0 * log(2.0) / log(c) * 4.0 / 3.0);
    return w > (double)(1 << 20) ? 0 : (int64_t)w;
}

// the split keys: plan, parts (one wave per 64 parts), check and reruns, on
// stream s; with_long: the long keys' waves in the parts' launch
// (td_ema_long_parts_kernel)
static int td_spec_launch(const double* values, const int64_t* seg_off, const double* init, double a,
                          double one_minus_a, double* out, const int64_t* long_idx, int64_t n_long, int64_t n_values,
                          int64_t warm, void* temp, hipStream_t s, bool with_long) {
    int64_t* hdr = static_cast<int64_t*>(temp);
    SpecPlanEntry* plan = reinterpret_cast<SpecPlanEntry*>(hdr + kSpecHdr);
    double* guess = reinterpret_cast<double*>(plan + std::max<int64_t>(n_long, 1));
    const int64_t parts = n_values / kSpecLen + n_long + 1;
    double* fin = guess + parts;
    const int warm16 = (int)((warm + kTdChunk - 1) / kTdChunk * kTdChunk);
    const hipError_t me = hipMemsetAsync(hdr, 0, sizeof(int64_t) * kSpecHdr, s);
    if (me != hipSuccess) return status(me);
    td_spec_select_kernel<<<blocks_for(n_long), kBlock, 0, s>>>(seg_off, long_idx, n_long, kSpecMinWarms * warm, hdr,
                                                                 plan);
    int rc = launched();
    if (rc != OTH_OK) return rc;
    td_spec_plan_kernel<<<1, kPlanThreads, 0, s>>>(hdr, plan, parts);
    rc = launched();
    if (rc != OTH_OK) return rc;
    const int64_t items = std::min<int64_t>(parts / kSpecLanes + n_long, 1024);
    if (with_long)
        td_ema_long_parts_kernel<<<(unsigned)(n_long + items), 64, 0, s>>>(values, seg_off, init, a, one_minus_a, out,
                                                                            long_idx, warm, n_long, hdr, plan, guess,
                                                                            fin, warm16, items);
    else
        td_spec_parts_kernel<<<(unsigned)items, kSpecLanes, 0, s>>>(values, seg_off, init, a, one_minus_a, hdr, plan,
                                                                     guess, fin, warm16);
    rc = launched();
    if (rc != OTH_OK) return rc;
    td_spec_fix_kernel<<<(unsigned)std::min<int64_t>(n_long, 256), kSpecLanes, 0, s>>>(values, seg_off, init, a,
                                                                                         one_minus_a, hdr, plan, guess,
                                                                                         fin, out);
    return launched();
}

int oth_td_ema_split(const double* values, const int64_t* seg_off, const double* init, double a,
                     double one_minus_a, double* out, int64_t n_seg, int64_t long_min, const int64_t* long_idx,
                     int64_t n_long, int64_t n_values, void* temp, size_t* temp_bytes, void* stream) {
    if (n_seg < 0 || long_min < 1 || n_long < 0 || n_long > n_seg || n_values < 0 || !temp_bytes ||
        (n_seg > 0 && (!values || !seg_off || !out)) || (n_long > 0 && !long_idx))
        return OTH_EINVAL;
    const int64_t warm = td_spec_warm(one_minus_a);
    const size_t need = warm > 0 && n_long > 0 ? spec_scratch_bytes(n_long, n_values) : 0;
    if (!temp) {  // size query: no work, no launch
        *temp_bytes = need;
        return OTH_OK;
    }
    if (*temp_bytes < need) return OTH_EINVAL;
    if (n_seg == 0) return OTH_OK;
    // the long keys (one wave each) and the split keys (plan, parts, check and
    // reruns) on the device's two side streams, launched first, beside the
    // short keys' kernel on the caller's stream: the three write disjoint
    // outputs and read only what the caller's stream did before this call
    const hipStream_t s = (hipStream_t)stream;
    TdFork fork(s, n_long == 0 ? 0 : (warm > 0 ? 2 : 1));
    if (fork.rc != OTH_OK) return fork.rc;
    // on one stream (no fork), the long keys share the split keys' parts
    // launch (OTH_TD_EMA_MERGED=0 in the environment: separate launches, A/B)
    static const int merged_ok = env_int("OTH_TD_EMA_MERGED", 1);
    const bool split = n_long > 0 && warm > 0, merged = split && fork.n == 0 && merged_ok;
    int rc = OTH_OK;
    if (n_long > 0 && !merged) {
        td_ema_long_kernel<<<(unsigned)n_long, 64, 0, fork.side(0)>>>(values, seg_off, init, a, one_minus_a, out,
                                                                       long_idx, warm);
        rc = launched();
    }
    if (rc == OTH_OK && split) rc = td_spec_launch(values, seg_off, init, a, one_minus_a, out, long_idx, n_long,
                                                   n_values, warm, temp, fork.side(1), merged);
    if (rc != OTH_OK) return fork.join(rc);
    if (long_min <= 3 * kTdChunk)
        td_ema_kernel<true><<<blocks_for(n_seg), kBlock, 0, s>>>(values, seg_off, init, a, one_minus_a, out, n_seg,
                                                                 long_min);
    else
        td_ema_kernel<false><<<blocks_for(n_seg), kBlock, 0, s>>>(values, seg_off, init, a, one_minus_a, out, n_seg,
                                                                  long_min);
    return fork.join(launched());
}

int oth_rollout_grid(int policy, int64_t n) {
    if (n < 0 || policy < OTH_POLICY_RANDOM || policy > OTH_POLICY_EVAL) return OTH_EINVAL;
    DeviceState* ds = device_state();
    if (!ds) return status(hipErrorInvalidDevice);
    const Tuning& t = ds->tuning;
    const unsigned resident =
        policy == OTH_POLICY_RANDOM && n >= kBigLaunch ? t.random_big_blocks : t.resident_blocks[policy];
    return (int)std::min<int64_t>((n + kBlock - 1) / kBlock, (int64_t)resident);
}

int oth_sample_midgame(uint64_t seed, uint64_t index0, uint64_t* boards, uint8_t* turn, uint8_t* nturn,
                       uint8_t* move, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!boards || !turn || !move))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    sample_midgame_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(mix64(seed + GOLDEN64), index0, boards,
                                                                             turn, nturn, move, n);
    return launched();
}

}  // extern "C"
