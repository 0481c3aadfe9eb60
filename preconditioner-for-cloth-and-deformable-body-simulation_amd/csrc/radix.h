// radix.h -- the stable (key, int) radix sort every phase uses: 32-bit keys
// through rsort.hip (no decoupled look-back, see there), 64-bit keys (the
// Morton codes of Allocate) through rocprim.
//
// rocprim::radix_sort_pairs with MergeSortLimit = 0: always the onesweep
// algorithm (ceil(bits / 8) passes) above one block.  With its default config
// rocprim sorts up to 2^20 items with keys wider than 2 bytes by a block sort
// plus ~20 merge passes -- ~130 us per 1M-item sort on MI355X, where onesweep
// needs two or three ~25 us passes for the 10-20-bit keys sorted here.  Both
// are stable (ties keep input order), which every caller relies on.
#pragma once

#include <rocprim/device/device_radix_sort.hpp>

#include "mas_internal.h"

namespace mas {

using OnesweepAlways =
    rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;

template <class K>
int sort_pairs(mas_context* h, const K* kin, K* kout, const int* vin, int* vout, int n, int bits, hipStream_t s,
               const char* what) {
    if (n <= 0) return MAS_OK;
    // 32-bit keys: the look-back-free sort (rsort.hip) unless MAS_SORT=0
    if constexpr (sizeof(K) == 4)
        if (h->sortImpl)
            return rs_sort_pairs(h, reinterpret_cast<const unsigned*>(kin), reinterpret_cast<unsigned*>(kout), vin,
                                 vout, n, bits, s, what);
    size_t tmp = 0;
    rocprim::radix_sort_pairs<OnesweepAlways>(nullptr, tmp, kin, kout, vin, vout, (size_t)n, 0, bits, s);
    int rc = ensure(h, h->cubTemp, tmp);
    if (rc) return rc;
    return hip_check(
        h, rocprim::radix_sort_pairs<OnesweepAlways>(h->cubTemp.p, tmp, kin, kout, vin, vout, (size_t)n, 0, bits, s),
        what);
}

}  // namespace mas
