// The sort key of the TD state map's packed update words (include/othello.h
// OTH_TD_SKEY_BITS, round 5): the counts() tuple (discs, moves, regions a..h)
// numbered in an order-preserving mixed radix, so the grouping sort orders the
// words exactly as it would by their OTH_TD_KEY but over 36 bits, four radix
// passes of 9 bits instead of the 43-bit key's five.
//   * (discs d, moves m): m <= 64 - d (a legal move is an empty square), so the
//     pairs are numbered triangularly, tri(d) + m with tri(d) = sum over
//     d' < d of (65 - d') = 65 d - d (d - 1) / 2: 2,145 pairs in (d, m) order.
//   * regions a..h: each count 0..size, the digits of a mixed radix with bases
//     size + 1 = 5, 9, 5, 9, 9, 17, 5, 13, a most significant.
//   skey = ((tri(d) + m) * 5 + r_a) << 22 | (r_b..r_h in their mixed radix,
//          < 4,027,725 < 2^22)  <  10,725 * 2^22 < 2^36.
// Lexicographic tuple order == OTH_TD_KEY integer order == skey order.  The
// split at bit 22 keeps the decode in 32-bit arithmetic (no 64-bit division).
#pragma once
#include <stdint.h>

#include "../../include/othello.h"

namespace td_skey {
constexpr uint32_t kBase[8] = {5, 9, 5, 9, 9, 17, 5, 13};
constexpr int kLowBits = 22;
constexpr int kKeyShift[8] = {27, 23, 20, 16, 12, 7, 4, 0};  // OTH_TD_KEY region fields
static_assert(9u * 5 * 9 * 9 * 17 * 5 * 13 <= (1u << kLowBits), "low part");
static_assert((2145ull * 5) << kLowBits <= (1ull << OTH_TD_SKEY_BITS), "skey range");

__host__ __device__ __forceinline__ uint32_t tri(uint32_t d) { return 65u * d - (d * (d - 1u) >> 1); }

// d = discs, m = moves (<= 64 - d), r = the region counts a..h
__device__ __forceinline__ uint64_t encode(uint32_t d, uint32_t m, const uint32_t (&r)[8]) {
    uint32_t lo = r[1];
#pragma unroll
    for (int k = 2; k < 8; k++) lo = lo * kBase[k] + r[k];
    return ((uint64_t)((tri(d) + m) * kBase[0] + r[0]) << kLowBits) | lo;
}

// skey -> OTH_TD_KEY
__device__ __forceinline__ int64_t to_key(uint64_t s) {
    const uint32_t hi = (uint32_t)(s >> kLowBits);
    uint32_t lo = (uint32_t)s & ((1u << kLowBits) - 1u);
    const uint32_t t = hi / kBase[0], ra = hi - t * kBase[0];
    // d: the largest with tri(d) <= t, from the inverse of the parabola
    // (131 d - d^2) / 2 = t, then corrected for the float's rounding
    uint32_t d = (uint32_t)((131.0f - __builtin_sqrtf(fmaxf(17161.0f - 8.0f * (float)t, 0.0f))) * 0.5f);
    d = min(d, 64u);
    if (d < 64u && tri(d + 1u) <= t) d++;
    if (tri(d) > t) d--;
    const uint32_t m = t - tri(d);
    uint32_t klo = ra << kKeyShift[0];
#pragma unroll
    for (int i = 7; i > 1; i--) {
        const uint32_t q = lo / kBase[i];
        klo |= (lo - q * kBase[i]) << kKeyShift[i];
        lo = q;
    }
    klo |= lo << kKeyShift[1];
    return (int64_t)(((uint64_t)((d << 6) | m) << 30) | klo);
}
}  // namespace td_skey
