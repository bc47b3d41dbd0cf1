// td_table.hip — the TD state map's table work around the EMA
// (progress_position_moves_learn.py:37-62 applies a batch's updates key by key,
// in stream order, to the store):
//   oth_td_sort_pairs: the update stream's (key, value) pairs in key order,
//     stable, so each key's values stay in stream order;
//   oth_td_lookup: the batch's keys looked up in the key-sorted table (their
//     states before the batch);
//   oth_td_merge: the batch's updated keys merged into the key-sorted table;
//   oth_td_fit_moments: the sums of the learner's per-shard regression.
//
// The sort:
// rocPRIM's onesweep radix sort of the pairs themselves over the key's 43 bits
// (OTH_TD_KEY_BITS), in 5 passes of 9-bit digits; the packed words of the GPU
// books' path over their 36-bit sort key (OTH_TD_SKEY_BITS, td_skey.hpp; round
// 5), 4 passes.  Round 3's key spent 5 bits
// on every region count and took 54 bits, 6 passes: 1.93 ms for 32.2M pairs
// (the gfx950 default of 8 bits a pass took 7 passes, 2.11-2.13 ms,
// tools/diag/sort_bits.hip; 10 bits ran 3.58 ms, 11 do not fit the LDS).
// torch.sort of the keys with a permutation is 8 passes of (key, int64 index)
// pairs plus a gather of the values by that permutation (profiles/design_history_r01_r04.md §10).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "../../include/othello.h"
#include "td_skey.hpp"

// packed words seen with a turn_left beyond lam_pow's OTH_POS_STRIDE entries
// (not words oth_td_updates_packed wrote: a corrupt or foreign word array),
// counted by every reader since the last oth_td_word_errors reset
__device__ unsigned long long g_td_bad_words;
// a turn_left field as an index into lam_pow: clamped, so such a word never
// reads past the table, and counted, so it is reported instead of hidden
__device__ __forceinline__ uint32_t td_turn_clamp(uint32_t t) {
    if (t < (uint32_t)OTH_POS_STRIDE) return t;
    atomicAdd(&g_td_bad_words, 1ull);
    return (uint32_t)OTH_POS_STRIDE - 1u;
}
__device__ __forceinline__ uint32_t td_turn_idx(uint64_t w) {
    return td_turn_clamp((uint32_t)(w >> OTH_TD_PACK_TURN_SHIFT) & OTH_TD_PACK_TURN_MASK);
}

namespace {

// onesweep digit width, items per thread and block size (tuned, round 5:
// profiles/r05_notes.md)
constexpr unsigned kSortBits = 9, kSortIpt = 8, kSortBlock = 1024;
using SortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<kSortBlock, kSortIpt>,
                                        rocprim::kernel_config<kSortBlock, kSortIpt>, kSortBits,
                                        rocprim::block_radix_rank_algorithm::match>>;

// packed words -> (key, value): the value recomputed from the payload exactly
// as oth_td_updates computes it
__global__ __launch_bounds__(256) void td_unpack_kernel(const uint64_t* __restrict__ words,
                                                        const double* __restrict__ lam_pow,
                                                        int64_t* __restrict__ keys, double* __restrict__ values,
                                                        int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t w = words[i];
    const int vs = (int)(w >> OTH_TD_PACK_VALUE_SHIFT) - 64;
    keys[i] = td_skey::to_key(w & ((1ull << OTH_TD_SKEY_BITS) - 1));
    values[i] = (double)vs * lam_pow[td_turn_idx(w)];
}

// The grouping sort (oth_td_sort_packed / oth_td_sort_unpack) is rocPRIM's
// onesweep radix sort (SortConfig above): the one vendor kernel on a §8 path.
// Round 5 built and A/B'd an own onesweep for gfx950 (ballot ranking, LDS
// stage, decoupled look-back): correct but 1.00-1.04 ms per 32.2M words
// against rocPRIM's 0.82, and 0.80 even with the look-back removed (wrong
// output, timing only), so it was not shipped; round 6 removed it from the
// source (tools/diag/td_own_sort.patch restores it; profiles/r05_notes.md).

constexpr int kMergeBlock = 256;
constexpr int kMergeK = 8;                               // merged positions per thread
constexpr int kMergeTile = kMergeBlock * kMergeK;        // per block
constexpr int kLookupK = 8;
constexpr int kLookupTile = kMergeBlock * kLookupK;

// A merge tile's inputs into LDS: A[a0, a0 + na) then B[b0, b0 + n - na)
// (keys, and values when Av / sv are given), every load of the thread in
// flight before its first LDS store (round 5: the strided loops these replace
// waited for each load before issuing the next -- the merge and lookup ran at
// ~3 TB/s, latency-bound)
template <int K>
__device__ __forceinline__ void stage_tile(const int64_t* __restrict__ A, const double* __restrict__ Av, int64_t a0,
                                           int na, const int64_t* __restrict__ B, const double* __restrict__ Bv,
                                           int64_t b0, int n, int64_t* sk, double* sv) {
    int64_t kk[K];
    double vv[K];
#pragma unroll
    for (int q = 0; q < K; q++) {
        const int e = (int)threadIdx.x + q * kMergeBlock;
        kk[q] = 0;
        vv[q] = 0.0;
        if (e < na) {
            kk[q] = A[a0 + e];
            if (Av) vv[q] = Av[a0 + e];
        } else if (e < n) {
            kk[q] = B[b0 + (e - na)];
            if (Bv) vv[q] = Bv[b0 + (e - na)];
        }
    }
#pragma unroll
    for (int q = 0; q < K; q++) {
        const int e = (int)threadIdx.x + q * kMergeBlock;
        if (e < n) {
            sk[e] = kk[q];
            if (sv) sv[e] = vv[q];
        }
    }
}

// The merge-path splits of every tile, one thread each, in a kernel of their
// own (the partition step of a merge path): split[s] is the first i in
// [max(0, d - nB), min(d, nA)] with A[i] >= B[d - i - 1] for diagonal
// d = min(s * tile, nA + nB) (A[i] < B[d - i - 1] holds below it, fails from
// it on), by a binary search of ~log2(n) dependent loads.  Round 2 searched
// inside each tile's block, cooperatively (~4 rounds of 128 probes per end,
// to avoid one thread's chain of dependent loads): every probe a random line,
// ~2,000 per block, which made the HBM traffic of the lookup and the merge
// 3-4x their algorithmic bytes (profiles/r03_profile_summary.json before
// this change).  Here all the searches run at once, ~25 loads each.
// nB_dev (oth_td_lookup_dev): B's length read from device memory, clamped to
// [0, nB]; the grid is sized for nB
__device__ __forceinline__ int64_t dev_count(const int64_t* nB_dev, int64_t nB) {
    return nB_dev ? min(max(*nB_dev, (int64_t)0), nB) : nB;
}
__global__ __launch_bounds__(kMergeBlock) void td_splits_kernel(const int64_t* __restrict__ A, int64_t nA,
                                                                const int64_t* __restrict__ B, int64_t nB,
                                                                int64_t tile, int64_t nsplit,
                                                                int64_t* __restrict__ split,
                                                                const int64_t* __restrict__ nB_dev) {
    const int64_t t = (int64_t)blockIdx.x * kMergeBlock + threadIdx.x;
    if (t >= nsplit) return;
    nB = dev_count(nB_dev, nB);
    const int64_t d = min(t * tile, nA + nB);
    int64_t lo = d > nB ? d - nB : 0, hi = d < nA ? d : nA;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (A[mid] < B[d - mid - 1]) lo = mid + 1;
        else hi = mid;
    }
    split[t] = lo;
}

// Merge path over the table (A: old keys, unique, sorted) and the batch's keys
// (B: unique, sorted; their new values), one tile of the merged sequence per
// block.  A table key equal to a batch key comes right after it and is
// dropped; every other element lands at its merged position minus the drops
// before it, which are the hits among the batch keys taken so far:
//   hits_before(j) = j - new_before[j].
// The block finds its tile's ends in A and B (two cooperative searches), stages
// the tile's keys and values in LDS with coalesced loads, each thread finds its
// own 8 positions by a search in LDS and merges them into registers, and the
// block writes its outputs (one contiguous range) back through LDS, coalesced.
__global__ __launch_bounds__(kMergeBlock) void td_merge_kernel(const int64_t* __restrict__ A,
                                                               const double* __restrict__ Av, int64_t nA,
                                                               const int64_t* __restrict__ B,
                                                               const double* __restrict__ Bv,
                                                               const int64_t* __restrict__ new_before, int64_t nB,
                                                               const int64_t* __restrict__ split,
                                                               int64_t* __restrict__ out_k,
                                                               double* __restrict__ out_v) {
    __shared__ int64_t sk[kMergeTile];
    __shared__ double sv[kMergeTile];
    __shared__ unsigned long long range[2];  // min slot, max slot + 1 of the block's outputs
    __shared__ int64_t prev_s;               // the batch key before the tile's first
    const int tid = threadIdx.x;
    const int64_t d0 = (int64_t)blockIdx.x * kMergeTile;
    const int64_t d1 = d0 + kMergeTile < nA + nB ? d0 + kMergeTile : nA + nB;
    if (tid == 0) {
        range[0] = ~0ull;
        range[1] = 0;
    }
    const int64_t s0 = split[blockIdx.x], s1 = split[blockIdx.x + 1];  // the tile's ends in A
    const int64_t a0 = s0, b0 = d0 - a0;
    const int na = (int)(s1 - a0), nb = (int)(d1 - s1 - b0);
    const int n = na + nb;
    if (tid == 0) prev_s = b0 > 0 ? B[b0 - 1] : -1;
    stage_tile<kMergeK>(A, Av, a0, na, B, Bv, b0, n, sk, sv);
    __syncthreads();
    const int t0 = min(tid * kMergeK, n), t1 = min(t0 + kMergeK, n);
    int lo = t0 > nb ? t0 - nb : 0, hi = t0 < na ? t0 : na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sk[mid] < sk[na + t0 - mid - 1]) lo = mid + 1;
        else hi = mid;
    }
    int i = lo, j = t0 - lo;
    // the batch key before this thread's first (keys are >= 0: -1 matches
    // none): from LDS, the tile's first from prev_s (round 5: a global load
    // per thread on the merge's critical path)
    int64_t prev_b = t0 < t1 ? (j > 0 ? sk[na + j - 1] : prev_s) : -1;
    // (a caller's inconsistent new_before must not send a store out of bounds)
    const uint64_t n_out = (uint64_t)(nA + new_before[nB]);
    int64_t ok[kMergeK];
    double ov[kMergeK];
    uint64_t os[kMergeK];
    unsigned long long smin = ~0ull, smax = 0;
    // the merge walk first, recording each output's batch index; then the
    // new_before loads of all of them at once (in the walk they were one
    // dependent global load per step; round 4)
    // Branch-free (round 5: the branchy walk compiled to ~420 v_mov_b64 of
    // predicated state copies): the two heads ka / kb stay in registers, a
    // step takes the smaller (A only if strictly smaller: a batch key before
    // its table copy), reads the taken element's value and refills the taken
    // head from LDS.  Heads past their side read as INT64_MAX (keys are
    // below 2^43).
    int64_t bq[kMergeK];
    constexpr int64_t kEnd = INT64_MAX;
    int64_t ka = i < na ? sk[i] : kEnd, kb = j < nb ? sk[na + j] : kEnd;
#pragma unroll
    for (int q = 0; q < kMergeK; q++) {
        const bool valid = t0 + q < t1;
        const bool takeA = ka < kb;  // (a valid step has a head below kEnd)
        const int at = takeA ? i : na + j;
        const int64_t key = takeA ? ka : kb;
        ov[q] = sv[at];
        ok[q] = key;
        bq[q] = valid && !(takeA && key == prev_b) ? b0 + j : -1;  // a table copy of the batch key just taken: dropped
        if (valid) {
            prev_b = takeA ? prev_b : key;
            i += takeA;
            j += !takeA;
            const int nx = takeA ? i : na + j;
            const int64_t head = (takeA ? i < na : j < nb) ? sk[nx] : kEnd;
            ka = takeA ? head : ka;
            kb = takeA ? kb : head;
        }
    }
    int64_t nbq[kMergeK];
#pragma unroll
    for (int q = 0; q < kMergeK; q++) nbq[q] = bq[q] >= 0 ? new_before[bq[q]] : 0;
#pragma unroll
    for (int q = 0; q < kMergeK; q++) {
        os[q] = bq[q] >= 0 ? (uint64_t)(d0 + t0 + q - (bq[q] - nbq[q])) : ~0ull;
        if (os[q] >= n_out) os[q] = ~0ull;
        if (os[q] != ~0ull) {
            smin = min(smin, (unsigned long long)os[q]);
            smax = max(smax, (unsigned long long)os[q] + 1);
        }
    }
    if (smin != ~0ull) {
        atomicMin(&range[0], smin);
        atomicMax(&range[1], smax);
    }
    __syncthreads();  // every thread is done reading sk / sv
    const unsigned long long base = range[0], end = range[1];
    if (base == ~0ull) return;  // a tile whose only element was dropped
#pragma unroll
    for (int q = 0; q < kMergeK; q++) {
        if (os[q] == ~0ull) continue;
        sk[os[q] - base] = ok[q];
        sv[os[q] - base] = ov[q];
    }
    __syncthreads();
    const int cnt_out = (int)(end - base);  // <= kMergeTile: one slot per merged position at most
#pragma unroll
    for (int q = 0; q < kMergeK; q++) {
        const int k = tid + q * kMergeBlock;
        if (k < cnt_out) {
            out_k[base + k] = sk[k];
            out_v[base + k] = sv[k];
        }
    }
}

// The batch's keys (B) looked up in the table (A) by the same merge path:
// a batch key at merged position m has the m - j table keys below it taken
// before it, and is in the table iff the next table key equals it.  The
// tile's batch keys are one contiguous range of B: their init values and
// is_new flags are staged in LDS and written by the block with coalesced
// stores (a thread's own stores, 8 scattered bytes per lane per step, wrote
// ~5x the bytes they held).
__global__ __launch_bounds__(kMergeBlock) void td_lookup_kernel(const int64_t* __restrict__ A,
                                                                const double* __restrict__ Av, int64_t nA,
                                                                const int64_t* __restrict__ B, int64_t nB,
                                                                const int64_t* __restrict__ split,
                                                                double* __restrict__ init,
                                                                uint8_t* __restrict__ is_new,
                                                                const int64_t* __restrict__ nB_dev) {
    __shared__ int64_t sk[kLookupTile];
    __shared__ int shit[kLookupTile];  // a batch key's table entry relative to a0, or -1 (not in the table)
    const int tid = threadIdx.x;
    const int64_t d0 = (int64_t)blockIdx.x * kLookupTile;
    nB = dev_count(nB_dev, nB);
    if (d0 >= nA + nB) return;  // past the device count (a whole block: before any barrier)
    const int64_t d1 = d0 + kLookupTile < nA + nB ? d0 + kLookupTile : nA + nB;
    const int64_t s0 = split[blockIdx.x], s1 = split[blockIdx.x + 1];
    const int64_t a0 = s0, b0 = d0 - a0;
    const int na = (int)(s1 - a0), nb = (int)(d1 - s1 - b0);
    const int n = na + nb;
    stage_tile<kLookupK>(A, nullptr, a0, na, B, nullptr, b0, n, sk, nullptr);
    __syncthreads();
    const int t0 = min(tid * kLookupK, n), t1 = min(t0 + kLookupK, n);
    int lo = t0 > nb ? t0 - nb : 0, hi = t0 < na ? t0 : na;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sk[mid] < sk[na + t0 - mid - 1]) lo = mid + 1;
        else hi = mid;
    }
    int i = lo, j = t0 - lo;
    // branch-free walk, the two heads in registers (as td_merge_kernel)
    constexpr int64_t kEnd = INT64_MAX;
    int64_t ka = i < na ? sk[i] : kEnd, kb = j < nb ? sk[na + j] : kEnd;
#pragma unroll
    for (int q = 0; q < kLookupK; q++) {
        if (t0 + q >= t1) break;
        const bool takeA = ka < kb;
        if (!takeA) {
            // batch key b0 + j; the next table key is A[a0 + i] (past the tile: from HBM)
            const int64_t ai = a0 + i;
            const int64_t next = i < na ? ka : (ai < nA ? A[ai] : -1);
            shit[j] = next == kb ? i : -1;
        }
        i += takeA;
        j += !takeA;
        const int nx = takeA ? i : na + j;
        const int64_t head = (takeA ? i < na : j < nb) ? sk[nx] : kEnd;
        ka = takeA ? head : ka;
        kb = takeA ? kb : head;
    }
    __syncthreads();
    // the hits' values loaded here, all in flight at once, not one per step of
    // the merge loop above (round 4)
    // (unrolled: every hit's load in flight before the first store; round 5)
    double hv[kLookupK];
#pragma unroll
    for (int q = 0; q < kLookupK; q++) {
        const int k = tid + q * kMergeBlock;
        const int r = k < nb ? shit[k] : -1;
        hv[q] = r >= 0 ? Av[a0 + r] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kLookupK; q++) {
        const int k = tid + q * kMergeBlock;
        if (k < nb) {
            init[b0 + k] = hv[q];
            is_new[b0 + k] = shit[k] >= 0 ? 0 : 1;
        }
    }
}

// Moments of the learner's regression over one shard's states (a contiguous
// range of the key-sorted table: the phase is the key's top field).  x = the
// 9 counts() features after the phase, y = the state value.  Pass 1 (mean ==
// NULL): n, sum x, sum y.  Pass 2: the centred cross products sum (x - mx)(x -
// mx)^T (upper triangle, 45) and sum (x - mx)(y - my) (9).  Each block leaves
// its partial sums in its own row of `partials` (OTH_TD_FIT_COLS doubles); the
// caller adds the OTH_TD_FIT_BLOCKS rows, in a fixed order: deterministic.
constexpr int kFitBlock = 256;
// counts()[1..9] of an OTH_TD_KEY (include/othello.h layout)
__device__ __forceinline__ void td_features(int64_t k, double (&x)[9]) {
    constexpr int kShift[9] = {30, 27, 23, 20, 16, 12, 7, 4, 0}, kWidth[9] = {6, 3, 4, 3, 4, 4, 5, 3, 4};
#pragma unroll
    for (int f = 0; f < 9; f++) x[f] = (double)((k >> kShift[f]) & ((1 << kWidth[f]) - 1));
}
template <int NACC>
__device__ __forceinline__ void block_sum_to_row(double (&acc)[NACC], double* row, double* lds) {
    // wave sums by xor shuffles, then the block's waves through LDS
#pragma unroll
    for (int q = 0; q < NACC; q++) {
        double v = acc[q];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        acc[q] = v;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int q = 0; q < NACC; q++) lds[wave * NACC + q] = acc[q];
    __syncthreads();
    for (int q = threadIdx.x; q < NACC; q += blockDim.x) {
        double v = 0.0;
        for (int w = 0; w < kFitBlock / 64; w++) v += lds[w * NACC + q];
        row[q] = v;
    }
}
__global__ __launch_bounds__(kFitBlock) void td_fit_pass1_kernel(const int64_t* __restrict__ keys,
                                                                 const double* __restrict__ vals, int64_t n,
                                                                 double* __restrict__ partials) {
    __shared__ double lds[(kFitBlock / 64) * 11];
    double acc[11] = {};
    for (int64_t i = (int64_t)blockIdx.x * kFitBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kFitBlock) {
        double x[9];
        td_features(keys[i], x);
        acc[0] += 1.0;
#pragma unroll
        for (int f = 0; f < 9; f++) acc[1 + f] += x[f];
        acc[10] += vals[i];
    }
    block_sum_to_row(acc, partials + (int64_t)blockIdx.x * OTH_TD_FIT_COLS, lds);
}
__global__ __launch_bounds__(kFitBlock) void td_fit_pass2_kernel(const int64_t* __restrict__ keys,
                                                                 const double* __restrict__ vals, int64_t n,
                                                                 const double* __restrict__ mean,
                                                                 double* __restrict__ partials) {
    __shared__ double lds[(kFitBlock / 64) * 54];
    double mx[9];
#pragma unroll
    for (int f = 0; f < 9; f++) mx[f] = mean[f];
    const double my = mean[9];
    double acc[54] = {};
    for (int64_t i = (int64_t)blockIdx.x * kFitBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kFitBlock) {
        double x[9];
        td_features(keys[i], x);
#pragma unroll
        for (int f = 0; f < 9; f++) x[f] -= mx[f];
        const double y = vals[i] - my;
        int q = 0;
#pragma unroll
        for (int f = 0; f < 9; f++)
#pragma unroll
            for (int g = f; g < 9; g++) acc[q++] += x[f] * x[g];
#pragma unroll
        for (int f = 0; f < 9; f++) acc[45 + f] += x[f] * y;
    }
    block_sum_to_row(acc, partials + (int64_t)blockIdx.x * OTH_TD_FIT_COLS, lds);
}

// the tiles' merge-path splits (tiles + 1 of them) into the caller's scratch
hipError_t merge_splits(const int64_t* A, int64_t nA, const int64_t* B, int64_t nB, int64_t tile, int64_t tiles,
                        int64_t* split, hipStream_t stream, const int64_t* nB_dev = nullptr) {
    const int64_t ns = tiles + 1;
    td_splits_kernel<<<(unsigned)((ns + kMergeBlock - 1) / kMergeBlock), kMergeBlock, 0, stream>>>(A, nA, B, nB, tile,
                                                                                                  ns, split, nB_dev);
    return hipGetLastError();
}
// the split table's bytes for n merged positions in tiles of `tile` (0 when
// nothing is merged)
// ---- segments of the key-sorted update stream (oth_td_segments): where
// torch's unique_consecutive + cumsum + nonzero took ~0.37 ms per 32M
// updates (a reduce-by-key, a scan, a partition and their fills, and two
// host syncs), one wave streams 512 keys in 8 coalesced rounds of 64: a
// segment starts where a key differs from the one before (the lane's
// neighbour by a DPP shift, the round's first from the round before), a
// ballot and mbcnt place the starts.  A count pass and a write pass around a
// scan of the waves' counts (rocPRIM) keep the order; the long segments the
// same way, by a second ballot and scan.
// rounds of 64 words per wave: 8 (late round 5; tools/diag/td_ab.sh, two
// passes, count / write pass per 32.2M words: 4 rounds 78 / 137 us, 6: 75 /
// 134, 8: 71 / 133, 16: 79 / 137, 32: 103 / 153)
constexpr int kSegRounds = 8;
constexpr int kSegWaveKeys = 64 * kSegRounds;
constexpr int kSegBlock = 256;
constexpr int kSegWavesPerBlock = kSegBlock / 64;
// A segment that starts at i is long iff keys[i + long_min - 1] is its key
// (the keys are sorted), taken from the lane long_min - 1 places on in the
// wave's registers (this round's keys or the next round's, by __shfl; round
// 5: staged in LDS before, whose 35 KiB per block held the count pass to 4
// blocks per CU), or from memory for long_min > 65.  Both passes find starts and long starts; the count pass
// leaves the wave's two counts, the write pass (after their scans) places
// both in order.  (The long keys by atomic appends instead: 25k appends to
// one counter cost the write pass 83 -> 368 us.)
// WORDS (oth_td_segments_words, round 5): the input is the key-sorted packed
// words themselves, each read as its skey (the low OTH_TD_SKEY_BITS; ukeys get
// the OTH_TD_KEY), and the write pass also writes every update's value
// (oth_td_unpack's rule), so the sorted stream needs no separate unpack into a
// keys array and a values array.
template <bool WRITE, bool WORDS = false>
__global__ __launch_bounds__(kSegBlock) void td_seg_kernel(const int64_t* __restrict__ keys, int64_t n,
                                                           int64_t* __restrict__ wave_cnt,
                                                           int64_t* __restrict__ wave_lcnt,
                                                           int64_t* __restrict__ seg_off,
                                                           int64_t* __restrict__ ukeys, int64_t long_min,
                                                           int64_t* __restrict__ long_idx,
                                                           const double* __restrict__ lam_pow = nullptr,
                                                           double* __restrict__ values = nullptr) {
    constexpr int64_t kKeyMask = (1ll << OTH_TD_SKEY_BITS) - 1;
    auto key_of = [](int64_t x) { return WORDS ? (x & kKeyMask) : x; };
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * kSegWavesPerBlock + (threadIdx.x >> 6);
    const int64_t base = w * kSegWaveKeys;
    if (base >= n) return;  // wave-uniform
    // every round's key loaded before the first is used (kSegRounds + 1 loads in flight:
    // k[kSegRounds] is the next wave's first round)
    int64_t k[kSegRounds + 1];
    uint32_t payload[kSegRounds];  // WORDS, WRITE: the word's top 28 bits
#pragma unroll
    for (int r = 0; r <= kSegRounds; r++) {
        const int64_t i = base + r * 64 + lane;
        const int64_t x = i < n ? keys[i] : 0;
        k[r] = key_of(x);
        if (r < kSegRounds) payload[r] = (uint32_t)((uint64_t)x >> OTH_TD_PACK_TURN_SHIFT);
    }
    const int ahead = (int)long_min - 1;  // (wave-uniform)
    const bool by_shfl = ahead <= 64;
    const int src = (lane + ahead) & 63;
    int64_t prev_last = base > 0 ? key_of(keys[base - 1]) : 0;
    int64_t pos = WRITE ? wave_cnt[w] : 0, lpos = WRITE ? wave_lcnt[w] : 0;  // after the scans: the wave's firsts
#pragma unroll
    for (int r = 0; r < kSegRounds; r++) {
        const int64_t i = base + r * 64 + lane;
        if (WORDS && WRITE && i < n) {
            const int vs = (int)(payload[r] >> (OTH_TD_PACK_VALUE_SHIFT - OTH_TD_PACK_TURN_SHIFT)) - 64;
            values[i] = (double)vs * lam_pow[td_turn_clamp(payload[r] & OTH_TD_PACK_TURN_MASK)];
        }
        int64_t before = __shfl_up(k[r], 1);
        if (lane == 0) before = prev_last;
        const bool start = i < n && (i == 0 || k[r] != before);
        const int64_t e = i + long_min - 1;
        bool lng = false;
        if (by_shfl) {
            const int64_t here = __shfl(k[r], src), next = __shfl(k[r + 1], src);
            lng = start && e < n && (lane + ahead < 64 ? here : next) == k[r];
        } else {
            lng = start && e < n && key_of(keys[e]) == k[r];
        }
        const uint64_t m = __ballot(start), ml = __ballot(lng);
        if (WRITE && start) {
            const int64_t at =
                pos + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            seg_off[at] = i;
            ukeys[at] = WORDS ? td_skey::to_key((uint64_t)k[r]) : k[r];
            if (lng)
                long_idx[lpos + __builtin_amdgcn_mbcnt_hi((uint32_t)(ml >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)ml, 0u))] = at;
        }
        pos += __popcll(m);
        lpos += __popcll(ml);
        prev_last = __shfl(k[r], 63);
    }
    if (!WRITE && lane == 0) {
        wave_cnt[w] = pos;
        wave_lcnt[w] = lpos;
    }
}
template <bool WRITE>
__global__ __launch_bounds__(kSegBlock) void td_count_kernel(const uint8_t* __restrict__ flags, int64_t n,
                                                             int64_t* __restrict__ wave_cnt,
                                                             int64_t* __restrict__ before) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * kSegWavesPerBlock + (threadIdx.x >> 6);
    const int64_t base = w * kSegWaveKeys;
    if (base >= n) return;  // wave-uniform
    int64_t pos = WRITE ? wave_cnt[w] : 0;
#pragma unroll 4
    for (int r = 0; r < kSegRounds; r++) {
        const int64_t i = base + r * 64 + lane;
        const bool set = i < n && flags[i] != 0;
        const uint64_t m = __ballot(set);
        if (WRITE && i < n)
            before[i] = pos + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        pos += __popcll(m);
    }
    if (!WRITE && lane == 0) wave_cnt[w] = pos;
}
// after the exclusive scan of the waves' counts (wave_off): the total into
// *total, and end_slot_base[total] = n (if given)
__global__ void td_seg_finish_kernel(const int64_t* __restrict__ wave_cnt, const int64_t* __restrict__ wave_off,
                                     int64_t n_waves, int64_t n, int64_t* __restrict__ end_slot_base,
                                     int64_t* __restrict__ total_out) {
    const int64_t total = n_waves > 0 ? wave_off[n_waves - 1] + wave_cnt[n_waves - 1] : 0;
    *total_out = total;
    if (end_slot_base) end_slot_base[total] = n;
}
// the waves' counts -> their exclusive prefixes (rocPRIM's device scan), then
// the finish kernel; temp: [wave_cnt | wave_off | rocPRIM's scratch]
hipError_t seg_scan(int64_t* wave_cnt, int64_t* wave_off, int64_t n_waves, int64_t n, int64_t* end_slot_base,
                    int64_t* total_out, void* scan_temp, size_t scan_bytes, hipStream_t st) {
    if (n_waves > 0) {
        const hipError_t e = rocprim::exclusive_scan(scan_temp, scan_bytes, wave_cnt, wave_off, (int64_t)0,
                                                     (size_t)n_waves, rocprim::plus<int64_t>(), st);
        if (e != hipSuccess) return e;
    }
    td_seg_finish_kernel<<<1, 1, 0, st>>>(wave_cnt, wave_off, n_waves, n, end_slot_base, total_out);
    return hipGetLastError();
}
size_t seg_scan_bytes(int64_t n_waves) {
    size_t b = 0;
    const int64_t* nul = nullptr;
    (void)rocprim::exclusive_scan(nullptr, b, nul, (int64_t*)nullptr, (int64_t)0, (size_t)(n_waves > 0 ? n_waves : 1),
                                  rocprim::plus<int64_t>());
    return b;
}

size_t split_bytes(int64_t n_old, int64_t n_upd, int64_t tile) {
    if (n_upd <= 0) return 0;
    return (size_t)((n_old + n_upd + tile - 1) / tile + 1) * sizeof(int64_t);
}

}  // namespace

extern "C" {

int oth_td_fit_moments(const int64_t* keys, const double* values, int64_t n, const double* mean,
                       double* partials, void* stream) {
    if (n < 0 || !partials || (n > 0 && (!keys || !values))) return OTH_EINVAL;
    if (mean)
        td_fit_pass2_kernel<<<OTH_TD_FIT_BLOCKS, kFitBlock, 0, (hipStream_t)stream>>>(keys, values, n, mean,
                                                                                      partials);
    else
        td_fit_pass1_kernel<<<OTH_TD_FIT_BLOCKS, kFitBlock, 0, (hipStream_t)stream>>>(keys, values, n, partials);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OTH_OK : -(int)e;
}

static int td_lookup(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                     int64_t n_upd, const int64_t* n_upd_dev, double* init, uint8_t* is_new, void* temp,
                     size_t* temp_bytes, void* stream) {
    if (n_old < 0 || n_upd < 0 || !temp_bytes) return OTH_EINVAL;
    const size_t need = split_bytes(n_old, n_upd, kLookupTile);
    if (!temp) {  // size query: no work, no launch
        *temp_bytes = need;
        return OTH_OK;
    }
    if ((n_old > 0 && (!old_keys || !old_vals)) || (n_upd > 0 && (!upd_keys || !init || !is_new)) ||
        *temp_bytes < need)
        return OTH_EINVAL;
    if (n_upd == 0) return OTH_OK;
    const int64_t n = n_old + n_upd;
    const int64_t tiles = (n + kLookupTile - 1) / kLookupTile;
    int64_t* split = static_cast<int64_t*>(temp);
    hipError_t e =
        merge_splits(old_keys, n_old, upd_keys, n_upd, kLookupTile, tiles, split, (hipStream_t)stream, n_upd_dev);
    if (e != hipSuccess) return -(int)e;
    td_lookup_kernel<<<(unsigned)tiles, kMergeBlock, 0, (hipStream_t)stream>>>(old_keys, old_vals, n_old, upd_keys,
                                                                              n_upd, split, init, is_new, n_upd_dev);
    e = hipGetLastError();
    return e != hipSuccess ? -(int)e : OTH_OK;
}
int oth_td_lookup(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                  int64_t n_upd, double* init, uint8_t* is_new, void* temp, size_t* temp_bytes, void* stream) {
    return td_lookup(old_keys, old_vals, n_old, upd_keys, n_upd, nullptr, init, is_new, temp, temp_bytes, stream);
}
int oth_td_lookup_dev(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                      int64_t n_upd_max, const int64_t* n_upd_dev, double* init, uint8_t* is_new, void* temp,
                      size_t* temp_bytes, void* stream) {
    if (temp && n_upd_max > 0 && !n_upd_dev) return OTH_EINVAL;
    return td_lookup(old_keys, old_vals, n_old, upd_keys, n_upd_max, n_upd_dev, init, is_new, temp, temp_bytes,
                     stream);
}

// split_ready: the merge path's splits already in place (a preceding lookup's
// scratch, oth_td_merge_after_lookup); else computed into temp
static int td_merge(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                    const double* upd_vals, const int64_t* new_before, int64_t n_upd, int64_t* out_keys,
                    double* out_vals, void* temp, const int64_t* split_ready, void* stream) {
    const int64_t n = n_old + n_upd;
    if (n == 0) return OTH_OK;
    if (n_upd == 0) {  // the table unchanged (new_before may be NULL: the kernel reads it)
        hipError_t e = hipMemcpyAsync(out_keys, old_keys, (size_t)n_old * sizeof(int64_t), hipMemcpyDeviceToDevice,
                                      (hipStream_t)stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(out_vals, old_vals, (size_t)n_old * sizeof(double), hipMemcpyDeviceToDevice,
                               (hipStream_t)stream);
        return e == hipSuccess ? OTH_OK : -(int)e;
    }
    const int64_t tiles = (n + kMergeTile - 1) / kMergeTile;
    const int64_t* split = split_ready;
    if (!split) {
        int64_t* s = static_cast<int64_t*>(temp);
        const hipError_t e = merge_splits(old_keys, n_old, upd_keys, n_upd, kMergeTile, tiles, s, (hipStream_t)stream);
        if (e != hipSuccess) return -(int)e;
        split = s;
    }
    td_merge_kernel<<<(unsigned)tiles, kMergeBlock, 0, (hipStream_t)stream>>>(
        old_keys, old_vals, n_old, upd_keys, upd_vals, new_before, n_upd, split, out_keys, out_vals);
    const hipError_t e = hipGetLastError();
    return e != hipSuccess ? -(int)e : OTH_OK;
}
int oth_td_merge(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                 const double* upd_vals, const int64_t* new_before, int64_t n_upd, int64_t* out_keys,
                 double* out_vals, void* temp, size_t* temp_bytes, void* stream) {
    if (n_old < 0 || n_upd < 0 || !temp_bytes) return OTH_EINVAL;
    const size_t need = split_bytes(n_old, n_upd, kMergeTile);
    if (!temp) {  // size query: no work, no launch
        *temp_bytes = need;
        return OTH_OK;
    }
    if ((n_old > 0 && (!old_keys || !old_vals)) || (n_upd > 0 && (!upd_keys || !upd_vals || !new_before)) ||
        (n_old + n_upd > 0 && (!out_keys || !out_vals)) || *temp_bytes < need)
        return OTH_EINVAL;
    return td_merge(old_keys, old_vals, n_old, upd_keys, upd_vals, new_before, n_upd, out_keys, out_vals, temp,
                    nullptr, stream);
}
// the lookup's tiles are the merge's, so its scratch holds the merge's splits
int oth_td_merge_after_lookup(const int64_t* old_keys, const double* old_vals, int64_t n_old, const int64_t* upd_keys,
                              const double* upd_vals, const int64_t* new_before, int64_t n_upd, int64_t* out_keys,
                              double* out_vals, const void* lookup_temp, void* stream) {
    static_assert(kMergeTile == kLookupTile, "the lookup's splits serve the merge");
    if (n_old < 0 || n_upd < 0 || (n_old > 0 && (!old_keys || !old_vals)) ||
        (n_upd > 0 && (!upd_keys || !upd_vals || !new_before || !lookup_temp)) ||
        (n_old + n_upd > 0 && (!out_keys || !out_vals)))
        return OTH_EINVAL;
    return td_merge(old_keys, old_vals, n_old, upd_keys, upd_vals, new_before, n_upd, out_keys, out_vals, nullptr,
                    static_cast<const int64_t*>(lookup_temp), stream);
}

int oth_td_sort_packed(const uint64_t* words_in, uint64_t* words_out, int64_t n, void* temp, size_t* temp_bytes,
                       void* stream) {
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    if (!temp) {  // size query: no work, no launch
        size_t bytes = 0;
        const hipError_t e = rocprim::radix_sort_keys<SortConfig>(nullptr, bytes, words_in, words_out, (size_t)n,
                                                                  0, OTH_TD_SKEY_BITS, (hipStream_t)stream);
        *temp_bytes = bytes;
        return e == hipSuccess ? OTH_OK : -(int)e;
    }
    if (n > 0 && (!words_in || !words_out)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    size_t bytes = *temp_bytes;
    const hipError_t e = rocprim::radix_sort_keys<SortConfig>(temp, bytes, words_in, words_out, (size_t)n,
                                                              0, OTH_TD_SKEY_BITS, (hipStream_t)stream);
    return e == hipSuccess ? OTH_OK : -(int)e;
}

int oth_td_sort_unpack(const uint64_t* words_in, const double* lam_pow, int64_t* keys, double* values, int64_t n,
                       void* temp, size_t* temp_bytes, void* stream) {
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    // rocPRIM's sort of the words into the scratch, then the unpack kernel
    size_t sort_bytes = 0;
    hipError_t e = rocprim::radix_sort_keys<SortConfig>(nullptr, sort_bytes, words_in, (uint64_t*)nullptr, (size_t)n,
                                                        0, OTH_TD_SKEY_BITS, (hipStream_t)stream);
    if (e != hipSuccess) return -(int)e;
    sort_bytes = (sort_bytes + 255) / 256 * 256;
    const size_t need = sort_bytes + (size_t)std::max<int64_t>(n, 1) * sizeof(uint64_t);
    if (!temp) {  // size query: no work, no launch
        *temp_bytes = need;
        return OTH_OK;
    }
    if (n > 0 && (!words_in || !lam_pow || !keys || !values ||
                  reinterpret_cast<const void*>(words_in) == reinterpret_cast<const void*>(keys)))
        return OTH_EINVAL;
    if (n >= (1ll << 32)) return OTH_EINVAL;  // 32-bit counts
    if (*temp_bytes < need) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    uint64_t* sorted = reinterpret_cast<uint64_t*>(static_cast<char*>(temp) + sort_bytes);
    e = rocprim::radix_sort_keys<SortConfig>(temp, sort_bytes, words_in, sorted, (size_t)n, 0, OTH_TD_SKEY_BITS,
                                             (hipStream_t)stream);
    if (e != hipSuccess) return -(int)e;
    td_unpack_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(sorted, lam_pow, keys, values, n);
    e = hipGetLastError();
    return e == hipSuccess ? OTH_OK : -(int)e;
}

}  // extern "C"
namespace {
template <bool WORDS>
int td_segments(const int64_t* keys, int64_t n, int64_t long_min, int64_t* seg_off, int64_t* ukeys, int64_t* long_idx,
                int64_t* counts, const double* lam_pow, double* values, void* temp, size_t* temp_bytes, void* stream) {
    if (n < 0 || long_min < 1 || !temp_bytes) return OTH_EINVAL;
    const int64_t n_waves = (n + kSegWaveKeys - 1) / kSegWaveKeys, slots = n_waves > 0 ? n_waves : 1;
    const size_t scan_bytes = seg_scan_bytes(n_waves);
    const size_t head = (4 * (size_t)slots * sizeof(int64_t) + 255) / 256 * 256;  // rocPRIM's scratch 256-B aligned
    const size_t need = head + scan_bytes;
    if (!temp) {  // size query: no work, no launch
        *temp_bytes = need;
        return OTH_OK;
    }
    if (!seg_off || !counts || (n > 0 && (!keys || !ukeys || !long_idx)) || *temp_bytes < need) return OTH_EINVAL;
    if (WORDS && n > 0 && (!lam_pow || !values)) return OTH_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    int64_t* wave_cnt = static_cast<int64_t*>(temp);
    int64_t* wave_off = wave_cnt + slots;
    int64_t* wave_lcnt = wave_off + slots;
    int64_t* wave_loff = wave_lcnt + slots;
    void* scan_temp = static_cast<char*>(temp) + head;
    const unsigned blocks = (unsigned)((n_waves + kSegWavesPerBlock - 1) / kSegWavesPerBlock);
    if (n > 0)
        td_seg_kernel<false, WORDS><<<blocks, kSegBlock, 0, st>>>(keys, n, wave_cnt, wave_lcnt, seg_off, ukeys,
                                                                  long_min, long_idx);
    hipError_t e = seg_scan(wave_cnt, wave_off, n_waves, n, seg_off, counts, scan_temp, scan_bytes, st);
    if (e == hipSuccess) e = seg_scan(wave_lcnt, wave_loff, n_waves, n, nullptr, counts + 1, scan_temp, scan_bytes, st);
    if (e != hipSuccess) return -(int)e;
    if (n > 0)
        td_seg_kernel<true, WORDS><<<blocks, kSegBlock, 0, st>>>(keys, n, wave_off, wave_loff, seg_off, ukeys,
                                                                 long_min, long_idx, lam_pow, values);
    e = hipGetLastError();
    return e == hipSuccess ? OTH_OK : -(int)e;
}
}  // namespace
extern "C" {

int oth_td_segments(const int64_t* keys, int64_t n, int64_t long_min, int64_t* seg_off, int64_t* ukeys,
                    int64_t* long_idx, int64_t* counts, void* temp, size_t* temp_bytes, void* stream) {
    return td_segments<false>(keys, n, long_min, seg_off, ukeys, long_idx, counts, nullptr, nullptr, temp,
                              temp_bytes, stream);
}

int oth_td_segments_words(const uint64_t* words, const double* lam_pow, int64_t n, int64_t long_min, int64_t* seg_off,
                          int64_t* ukeys, int64_t* long_idx, int64_t* counts, double* values, void* temp,
                          size_t* temp_bytes, void* stream) {
    return td_segments<true>(reinterpret_cast<const int64_t*>(words), n, long_min, seg_off, ukeys, long_idx, counts,
                             lam_pow, values, temp, temp_bytes, stream);
}

int oth_td_new_before(const uint8_t* is_new, int64_t n, int64_t* new_before, void* temp, size_t* temp_bytes,
                      void* stream) {
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    const int64_t n_waves = (n + kSegWaveKeys - 1) / kSegWaveKeys, slots = n_waves > 0 ? n_waves : 1;
    const size_t scan_bytes = seg_scan_bytes(n_waves);
    const size_t head = (2 * (size_t)slots * sizeof(int64_t) + 2 * sizeof(int64_t) + 255) / 256 * 256;
    const size_t need = head + scan_bytes;
    if (!temp) {  // size query: no work, no launch
        *temp_bytes = need;
        return OTH_OK;
    }
    if (!new_before || (n > 0 && !is_new) || *temp_bytes < need) return OTH_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    int64_t* wave_cnt = static_cast<int64_t*>(temp);
    int64_t* wave_off = wave_cnt + slots;
    int64_t* counts = wave_off + slots;  // [total, unused]
    const unsigned blocks = (unsigned)((n_waves + kSegWavesPerBlock - 1) / kSegWavesPerBlock);
    if (n > 0) td_count_kernel<false><<<blocks, kSegBlock, 0, st>>>(is_new, n, wave_cnt, new_before);
    hipError_t e = seg_scan(wave_cnt, wave_off, n_waves, n, nullptr, counts, static_cast<char*>(temp) + head,
                            scan_bytes, st);  // counts[0] = the total
    if (e != hipSuccess) return -(int)e;
    if (n > 0) td_count_kernel<true><<<blocks, kSegBlock, 0, st>>>(is_new, n, wave_off, new_before);
    e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(new_before + n, counts, sizeof(int64_t), hipMemcpyDeviceToDevice, st);
    return e == hipSuccess ? OTH_OK : -(int)e;
}

int oth_td_word_errors(uint64_t* count, int reset, void* stream) {
    if (!count) return OTH_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    void* dev = nullptr;
    hipError_t e = hipGetSymbolAddress(&dev, HIP_SYMBOL(g_td_bad_words));
    if (e == hipSuccess) e = hipMemcpyAsync(count, dev, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess && reset) e = hipMemsetAsync(dev, 0, sizeof(uint64_t), st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e == hipSuccess ? OTH_OK : -(int)e;
}

int oth_td_unpack(const uint64_t* words, const double* lam_pow, int64_t* keys, double* values, int64_t n,
                  void* stream) {
    if (n < 0 || (n > 0 && (!words || !lam_pow || !keys || !values))) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    td_unpack_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(words, lam_pow, keys, values, n);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OTH_OK : -(int)e;
}

int oth_td_sort_pairs(const int64_t* keys_in, const double* vals_in, int64_t* keys_out, double* vals_out, int64_t n,
                      void* temp, size_t* temp_bytes, void* stream) {
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    // the keys are non-negative and below 2^OTH_TD_KEY_BITS: as unsigned words
    // their order is the signed order, and the bits above are all zero
    const uint64_t* kin = reinterpret_cast<const uint64_t*>(keys_in);
    uint64_t* kout = reinterpret_cast<uint64_t*>(keys_out);
    if (!temp) {  // size query: no work, no launch
        size_t bytes = 0;
        const hipError_t e = rocprim::radix_sort_pairs<SortConfig>(nullptr, bytes, kin, kout, vals_in, vals_out, (size_t)n, 0,
                                                       OTH_TD_KEY_BITS, (hipStream_t)stream);
        *temp_bytes = bytes;
        return e == hipSuccess ? OTH_OK : -(int)e;
    }
    if (n > 0 && (!keys_in || !vals_in || !keys_out || !vals_out)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    size_t bytes = *temp_bytes;
    const hipError_t e = rocprim::radix_sort_pairs<SortConfig>(temp, bytes, kin, kout, vals_in, vals_out, (size_t)n, 0,
                                                   OTH_TD_KEY_BITS, (hipStream_t)stream);
    return e == hipSuccess ? OTH_OK : -(int)e;
}

}  // extern "C"
