// othello.hip — MI355X (gfx950) kernels + C-ABI for the batched Othello env.
//
// Replaces the step path of ysnrkdm/subproc board.py:
//   puttables / n_puttable_for  (board.py:46-55)   -> moves()      Kogge-Stone fills
//   put / put_s                 (board.py:161-209) -> flips()      Kogge-Stone fills
//   is_game_over                (board.py:57-58)   -> two-pass rule in the rollout loop
//   n_black / n_white + result  (board.py:37-41, game_runner.py:194-199)
//   play loop                   (game_runner.py:165-201) -> rollout_kernel
//
// Design: one game per lane, state in VGPRs as two uint64 bitboards
// (mover P, opponent O); pure integer/bitwise VALU work, no LDS tables, no MFMA.
// Rollouts keep every lane busy by refilling finished lanes from a per-wave game
// range with __ballot + mbcnt (wavefront compaction), and reduce the win/score
// histogram in LDS before one global atomic per bin per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/othello.h"

#define OTH_VERSION "subproc_amd 0.1.0 gfx950"

namespace {

typedef uint64_t u64;
typedef uint32_t u32;

constexpr u64 NOT_A = 0xFEFEFEFEFEFEFEFEull;  // clears file a (x = 0): destination mask for +x moves
constexpr u64 NOT_H = 0x7F7F7F7F7F7F7F7Full;  // clears file h (x = 7): destination mask for -x moves
constexpr u64 ALL = ~0ull;
constexpr u64 OPEN_BLACK = 0x0000000810000000ull;  // e4, d5  (board.py:25)
constexpr u64 OPEN_WHITE = 0x0000001008000000ull;  // d4, e5  (board.py:24)
constexpr int kBlock = 256;

// ---------------------------------------------------------------------------
// directional shifts: L = toward higher squares.  The 8 rays of board.py:9-17:
//   R (+1,0)=<<1 NOT_A   L (-1,0)=>>1 NOT_H   D (0,+1)=<<8   U (0,-1)=>>8
//   RD(+1,+1)=<<9 NOT_A  LD(-1,+1)=<<7 NOT_H  RU(+1,-1)=>>7 NOT_A  LU(-1,-1)=>>9 NOT_H
// ---------------------------------------------------------------------------
template <int S, bool L>
__device__ __forceinline__ u64 sh(u64 x) {
    return L ? (x << S) : (x >> S);
}

// Kogge-Stone occluded fill of `gen` through `pro` along one direction
// (3 doubling steps cover the 6-square maximum run).
template <int S, bool L>
__device__ __forceinline__ u64 ks_fill(u64 gen, u64 pro) {
    gen |= pro & sh<S, L>(gen);
    pro &= sh<S, L>(pro);
    gen |= pro & sh<2 * S, L>(gen);
    pro &= sh<2 * S, L>(pro);
    gen |= pro & sh<4 * S, L>(gen);
    return gen;
}

// legal squares for mover P in one direction: empty squares reached by a run
// of >=1 opponent discs that starts next to a P disc
template <int S, bool L, u64 M>
__device__ __forceinline__ u64 moves_dir(u64 P, u64 O, u64 E) {
    const u64 g = ks_fill<S, L>(P, O & M);
    return sh<S, L>(g & O) & M & E;
}

__device__ __forceinline__ u64 moves(u64 P, u64 O) {
    const u64 E = ~(P | O);
    u64 m = moves_dir<1, true, NOT_A>(P, O, E);
    m |= moves_dir<1, false, NOT_H>(P, O, E);
    m |= moves_dir<8, true, ALL>(P, O, E);
    m |= moves_dir<8, false, ALL>(P, O, E);
    m |= moves_dir<9, true, NOT_A>(P, O, E);
    m |= moves_dir<7, true, NOT_H>(P, O, E);
    m |= moves_dir<7, false, NOT_A>(P, O, E);
    m |= moves_dir<9, false, NOT_H>(P, O, E);
    return m;
}

// discs flipped by placing bit `mv` for mover P: the run of O from mv along a
// ray counts only if the square after it holds P (board.py:124-139)
template <int S, bool L, u64 M>
__device__ __forceinline__ u64 flips_dir(u64 mv, u64 P, u64 O) {
    const u64 g = ks_fill<S, L>(mv, O & M);
    return (sh<S, L>(g) & M & P) ? (g & O) : 0ull;
}

__device__ __forceinline__ u64 flips(u64 mv, u64 P, u64 O) {
    u64 f = flips_dir<1, true, NOT_A>(mv, P, O);
    f |= flips_dir<1, false, NOT_H>(mv, P, O);
    f |= flips_dir<8, true, ALL>(mv, P, O);
    f |= flips_dir<8, false, ALL>(mv, P, O);
    f |= flips_dir<9, true, NOT_A>(mv, P, O);
    f |= flips_dir<7, true, NOT_H>(mv, P, O);
    f |= flips_dir<7, false, NOT_A>(mv, P, O);
    f |= flips_dir<9, false, NOT_H>(mv, P, O);
    return f;
}

// index of the k-th set bit (LSB-first, 0-based) of x; requires k < popcount(x).
// Branch-free popcount bisection: identical cost in every lane.
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

// ---------------------------------------------------------------------------
// RNG spec (twins: oracle/othello_oracle.c, tests/golden/gen_golden.py)
// ---------------------------------------------------------------------------
constexpr u64 GOLDEN64 = 0x9E3779B97F4A7C15ull;
__host__ __device__ __forceinline__ u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ u32 mix32(u32 x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ u64 game_key(u64 S, u64 g) { return mix64(S + g * GOLDEN64); }
__device__ __forceinline__ u32 ply_rand(u64 key, u32 ply) {
    return mix32((u32)key ^ mix32((u32)(key >> 32) + ply));
}
__device__ __forceinline__ u32 pick(u64 key, u32 ply, u32 n) { return __umulhi(ply_rand(key, ply), n); }

// 1-ply greedy: legal move minimising the opponent's mobility on the child,
// ties -> lowest square (first in puttables order)
__device__ __forceinline__ u32 greedy_move(u64 legal, u64 P, u64 O) {
    u32 best = 64, bestv = 1000;
    while (legal) {
        const u32 sq = (u32)__ffsll((unsigned long long)legal) - 1u;
        const u64 mv = 1ull << sq;
        legal &= legal - 1;
        const u64 f = flips(mv, P, O);
        const u32 v = (u32)__popcll(moves(O & ~f, P | f | mv));
        if (v < bestv) {
            bestv = v;
            best = sq;
        }
    }
    return best;
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

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

__global__ __launch_bounds__(kBlock) void legal_kernel(const u64* __restrict__ boards,
                                                       const uint8_t* __restrict__ turn, u64* __restrict__ legal,
                                                       int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(boards)[i];
    const u32 t = turn[i];
    u64 m = 0;
    if (t == OTH_BLACK) m = moves(b.x, b.y);
    else if (t == OTH_WHITE) m = moves(b.y, b.x);
    legal[i] = m;
}

__global__ __launch_bounds__(kBlock) void step_kernel(const u64* boards_in,
                                                      const uint8_t* turn_in,
                                                      const uint8_t* __restrict__ move, u64* boards_out,
                                                      uint8_t* turn_out, u64* __restrict__ flips_out,
                                                      u64* __restrict__ legal_next, int8_t* __restrict__ ret_out,
                                                      uint8_t* __restrict__ nturn, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(boards_in)[i];
    const u32 t = turn_in[i];
    const u32 mvc = move[i];
    const bool valid_turn = (t == OTH_BLACK) | (t == OTH_WHITE);
    const bool black = t == OTH_BLACK;
    u64 P = black ? b.x : b.y;
    u64 O = black ? b.y : b.x;
    u64 f = 0;
    int r = -1;
    if (valid_turn) {
        if (mvc == OTH_PASS) {
            r = 0;
        } else if (mvc < 64) {
            const u64 mv = 1ull << mvc;
            if (!((P | O) & mv)) {
                f = flips(mv, P, O);
                if (f) {
                    r = __popcll(f);
                    P |= f | mv;
                    O &= ~f;
                }
            }
        }
    }
    const bool moved = r >= 0;
    const u32 t_out = moved ? (t ^ 3u) : t;
    // mover after the step: O if the turn toggled
    if (legal_next) legal_next[i] = valid_turn ? (moved ? moves(O, P) : moves(P, O)) : 0ull;
    if (boards_out) {
        const u64 nb = black ? P : O, nw = black ? O : P;
        reinterpret_cast<ulonglong2*>(boards_out)[i] = make_ulonglong2(valid_turn ? nb : b.x, valid_turn ? nw : b.y);
    }
    if (turn_out) turn_out[i] = (uint8_t)t_out;
    if (flips_out) flips_out[i] = f;
    if (ret_out) ret_out[i] = (int8_t)r;
    if (nturn && moved) nturn[i] = (uint8_t)(nturn[i] + 1);
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
// rollout kernel: one game per lane, finished lanes refilled from the wave's
// contiguous game range via ballot + mbcnt, until the range is exhausted.
// ---------------------------------------------------------------------------
struct RolloutArgs {
    const u64* start;
    const uint8_t* start_turn;
    u64 seed_state;
    u64 game_id0;
    int policy;
    int n_random;
    u64* final_boards;
    int8_t* diff;
    uint8_t* plies;
    uint8_t* moves;
    long long* hist;
    int64_t n;
    int64_t games_per_wave;
};

__global__ __launch_bounds__(kBlock) void rollout_kernel(RolloutArgs a) {
    __shared__ unsigned long long hist_s[OTH_HIST_BINS];
    for (int k = threadIdx.x; k < OTH_HIST_BINS; k += kBlock) hist_s[k] = 0;
    __syncthreads();

    const int lane = lane_id();
    const int64_t wave = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const int64_t w_begin = wave * a.games_per_wave;
    const int64_t w_end = min(a.n, w_begin + a.games_per_wave);

    // per-lane game state
    u64 P = 0, O = 0, key = 0;
    u32 side = OTH_BLACK, ply = 0;
    bool passed = false;
    int64_t g = -1;
    bool active = false;
    u64 plies_sum = 0;

    int64_t next = w_begin;  // wave-uniform
    bool need = true;        // this lane needs a game
    for (;;) {
        // ---- refill lanes that need a game (wavefront compaction)
        const u64 want = __ballot(need);
        if (want) {
            const u32 rank = __popcll(want & ((1ull << lane) - 1ull));  // mbcnt
            if (need) {
                g = next + rank;
                active = g < w_end;
                need = false;
                if (active) {
                    key = game_key(a.seed_state, a.game_id0 + (u64)g);
                    ply = 0;
                    passed = false;
                    u64 bl = OPEN_BLACK, wh = OPEN_WHITE;
                    side = OTH_BLACK;
                    if (a.start) {
                        const ulonglong2 s = reinterpret_cast<const ulonglong2*>(a.start)[g];
                        bl = s.x;
                        wh = s.y;
                        side = a.start_turn ? a.start_turn[g] : OTH_BLACK;
                        side = side == OTH_WHITE ? OTH_WHITE : OTH_BLACK;
                    }
                    P = side == OTH_BLACK ? bl : wh;
                    O = side == OTH_BLACK ? wh : bl;
                    if (a.moves) {
                        uint4* mrec = reinterpret_cast<uint4*>(a.moves + g * OTH_MOVES_STRIDE);
#pragma unroll
                        for (int q = 0; q < OTH_MOVES_STRIDE / 16; q++) mrec[q] = make_uint4(~0u, ~0u, ~0u, ~0u);
                    }
                }
            }
            next += __popcll(want);
        }
        if (!__ballot(active)) break;
        if (!active) continue;  // (exec-masked; loop continues while any lane is active)

        const u64 legal = moves(P, O);
        if (legal == 0) {
            if (passed) {
                // terminal: both sides without a legal move (board.py:57-58)
                const u64 bl = side == OTH_BLACK ? P : O, wh = side == OTH_BLACK ? O : P;
                const int d = __popcll(bl) - __popcll(wh);
                if (a.final_boards) reinterpret_cast<ulonglong2*>(a.final_boards)[g] = make_ulonglong2(bl, wh);
                if (a.diff) a.diff[g] = (int8_t)d;
                if (a.plies) a.plies[g] = (uint8_t)ply;
                atomicAdd(&hist_s[d + 64], 1ull);
                atomicAdd(&hist_s[d > 0 ? 129 : (d < 0 ? 130 : 131)], 1ull);
                plies_sum += ply;
                need = true;
            } else {
                // mover must pass: tentatively hand the move over; the pass is
                // counted once the other side is found to have a move
                passed = true;
                const u64 t = P;
                P = O;
                O = t;
                side ^= 3u;
            }
            continue;
        }
        if (passed) {
            if (a.moves && ply < OTH_MOVES_STRIDE) a.moves[g * OTH_MOVES_STRIDE + ply] = OTH_PASS;
            ply++;
            passed = false;
        }
        u32 sq;
        if (a.policy == OTH_POLICY_GREEDY && (int)ply >= a.n_random) {
            sq = greedy_move(legal, P, O);
        } else {
            sq = kth_bit(legal, pick(key, ply, (u32)__popcll(legal)));
        }
        const u64 mv = 1ull << sq;
        const u64 f = flips(mv, P, O);
        if (a.moves && ply < OTH_MOVES_STRIDE) a.moves[g * OTH_MOVES_STRIDE + ply] = (uint8_t)sq;
        const u64 np = O & ~f;
        O = P | f | mv;
        P = np;
        side ^= 3u;
        ply++;
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
        const u64 key = game_key(S, i ^ (attempt << 48));
        const u32 target = 10 + pick(key, 200, 40);
        u64 P = OPEN_BLACK, O = OPEN_WHITE;
        u32 side = OTH_BLACK, ply = 0;
        for (;;) {
            const u64 legal = moves(P, O);
            if (legal == 0 && moves(O, P) == 0) break;  // is_game_over
            if (ply >= target && legal) {
                const u32 sq = kth_bit(legal, pick(key, ply, (u32)__popcll(legal)));
                reinterpret_cast<ulonglong2*>(boards)[j] =
                    side == OTH_BLACK ? make_ulonglong2(P, O) : make_ulonglong2(O, P);
                turn[j] = (uint8_t)side;
                if (nturn) nturn[j] = (uint8_t)ply;
                move[j] = (uint8_t)sq;
                return;
            }
            if (legal) {
                const u64 mv = 1ull << kth_bit(legal, pick(key, ply, (u32)__popcll(legal)));
                const u64 f = flips(mv, P, O);
                P |= f | mv;
                O &= ~f;
            }
            const u64 t = P;
            P = O;
            O = t;
            side ^= 3u;
            ply++;
        }
    }
}

inline int status(hipError_t e) { return e == hipSuccess ? OTH_OK : -(int)e; }
inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }
inline int launched() { return status(hipGetLastError()); }

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
    step_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(boards_in, turn_in, move, boards_out, turn_out,
                                                                   flips, legal_next, ret, nturn, n);
    return launched();
}

int oth_result(const uint64_t* boards, uint8_t* n_black, uint8_t* n_white, int8_t* diff, uint8_t* terminal,
               int64_t n, void* stream) {
    if (n < 0 || (n > 0 && !boards)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    result_kernel<<<blocks_for(n), kBlock, 0, (hipStream_t)stream>>>(boards, n_black, n_white, diff, terminal, n);
    return launched();
}

int oth_rollout(const uint64_t* start, const uint8_t* start_turn, uint64_t seed, uint64_t game_id0, int policy,
                int n_random, uint64_t* final_boards, int8_t* diff, uint8_t* plies, uint8_t* moves, int64_t* hist,
                int64_t n, void* stream) {
    if (n < 0 || (policy != OTH_POLICY_RANDOM && policy != OTH_POLICY_GREEDY)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    RolloutArgs a;
    a.start = start;
    a.start_turn = start_turn;
    a.seed_state = mix64(seed + GOLDEN64);
    a.game_id0 = game_id0;
    a.policy = policy;
    a.n_random = n_random;
    a.final_boards = final_boards;
    a.diff = diff;
    a.plies = plies;
    a.moves = moves;
    a.hist = (long long*)hist;
    a.n = n;
    // aim for ~16 waves per CU on 256 CUs, at least 64 games per wave
    const int64_t target_waves = 256 * 16;
    int64_t gpw = (n + target_waves - 1) / target_waves;
    if (gpw < 64) gpw = 64;
    a.games_per_wave = gpw;
    const int64_t waves = (n + gpw - 1) / gpw;
    const unsigned grid = (unsigned)((waves + (kBlock / 64) - 1) / (kBlock / 64));
    rollout_kernel<<<grid, kBlock, 0, (hipStream_t)stream>>>(a);
    return launched();
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
