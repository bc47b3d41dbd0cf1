// td_sort.hip — the TD state map's grouping sort (include/othello.h
// oth_td_sort_pairs): the update stream's (key, value) pairs in key order,
// stable, so each key's values stay in stream order (the learner applies a
// book's updates in order, progress_position_moves_learn.py:37-62).
//
// rocPRIM's onesweep radix sort of the pairs themselves over the key's 54 bits
// (OTH_TD_KEY_BITS): 7 8-bit digit passes of 16-byte pairs.  torch.sort of the
// keys with a permutation is 8 passes of (key, int64 index) pairs plus a gather
// of the values by that permutation.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <climits>
#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/othello.h"

extern "C" {

int oth_td_sort_pairs(const int64_t* keys_in, const double* vals_in, int64_t* keys_out, double* vals_out, int64_t n,
                      void* temp, size_t* temp_bytes, void* stream) {
    if (n < 0 || !temp_bytes) return OTH_EINVAL;
    // the keys are non-negative and below 2^OTH_TD_KEY_BITS: as unsigned words
    // their order is the signed order, and the bits above are all zero
    const uint64_t* kin = reinterpret_cast<const uint64_t*>(keys_in);
    uint64_t* kout = reinterpret_cast<uint64_t*>(keys_out);
    if (!temp) {  // size query: no work, no launch
        size_t bytes = 0;
        const hipError_t e = rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, vals_in, vals_out, (size_t)n, 0,
                                                       OTH_TD_KEY_BITS, (hipStream_t)stream);
        *temp_bytes = bytes;
        return e == hipSuccess ? OTH_OK : -(int)e;
    }
    if (n > 0 && (!keys_in || !vals_in || !keys_out || !vals_out)) return OTH_EINVAL;
    if (n == 0) return OTH_OK;
    size_t bytes = *temp_bytes;
    const hipError_t e = rocprim::radix_sort_pairs(temp, bytes, kin, kout, vals_in, vals_out, (size_t)n, 0,
                                                   OTH_TD_KEY_BITS, (hipStream_t)stream);
    return e == hipSuccess ? OTH_OK : -(int)e;
}

}  // extern "C"
