// The sort key of the TD state map's packed update words (include/othello.h
// OTH_TD_SKEY_BITS, round 5): the counts() tuple (discs, moves, regions a..h)
// numbered in an order-preserving mixed radix, so the grouping sort orders the
// words exactly as it would by their OTH_TD_KEY but over 36 bits, four radix
// passes of 9 bits instead of the 43-bit key's five.
//   * (discs d, moves m): m <= 64 - d (a legal move is an empty square), so the
//     pairs are numbered triangularly, tri(d) + m with tri(d) = sum over
//     d' < d of (65 - d') = 65 d - d (d - 1) / 2: 2,145 pairs in (d, m) order.
//   * regions a..h: each count 0..size, the digits of a mixed radix with bases
//     size + 1 = 5, 9, 5, 9, 9, 17, 5, 13 (product 20,138,625), a most
//     significant.
//   skey = (tri(d) + m) * 20,138,625 + regions  <  2,145 * 20,138,625 < 2^36.
// Lexicographic tuple order == OTH_TD_KEY integer order == skey order.
#pragma once
#include <stdint.h>

#include "../../include/othello.h"

namespace td_skey {
constexpr uint32_t kBase[8] = {5, 9, 5, 9, 9, 17, 5, 13};
constexpr uint64_t kRegions = 20138625ull;  // product of kBase
constexpr int kKeyShift[8] = {27, 23, 20, 16, 12, 7, 4, 0};  // OTH_TD_KEY region fields
static_assert(2145ull * kRegions <= (1ull << OTH_TD_SKEY_BITS), "skey range");

__host__ __device__ __forceinline__ uint32_t tri(uint32_t d) { return 65u * d - (d * (d - 1u) >> 1); }

// d = discs, m = moves (<= 64 - d), r = the region counts a..h
__device__ __forceinline__ uint64_t encode(uint32_t d, uint32_t m, const uint32_t (&r)[8]) {
    uint32_t x = r[0];
#pragma unroll
    for (int k = 1; k < 8; k++) x = x * kBase[k] + r[k];
    return (uint64_t)(tri(d) + m) * kRegions + x;
}

// skey -> OTH_TD_KEY
__device__ __forceinline__ int64_t to_key(uint64_t s) {
    const uint32_t t = (uint32_t)(s / kRegions);
    uint32_t x = (uint32_t)(s - (uint64_t)t * kRegions);
    uint32_t d = 0;  // the largest d with tri(d) <= t (tri increases on 0..64)
#pragma unroll
    for (uint32_t step = 64; step; step >>= 1)
        if (d + step <= 64u && tri(d + step) <= t) d += step;
    const uint32_t m = t - tri(d);
    uint64_t k = ((uint64_t)d << 36) | ((uint64_t)m << 30);
#pragma unroll
    for (int i = 7; i > 0; i--) {
        k |= (uint64_t)(x % kBase[i]) << kKeyShift[i];
        x /= kBase[i];
    }
    return (int64_t)(k | ((uint64_t)x << kKeyShift[0]));
}
}  // namespace td_skey
