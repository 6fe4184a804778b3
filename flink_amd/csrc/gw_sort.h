#pragma once
#include "gw_device.h"

namespace gw {
int64_t radix_sort_scratch_bytes(int64_t n);
// Sorts (k0, v0) by the low `bits` bits of the key; result in (k1, v1) if *result_in_alt.
hipError_t radix_sort_pairs(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, int64_t n, int bits,
                            void* scratch, hipStream_t s, int* result_in_alt);
hipError_t launch_iota(uint32_t* v, int64_t n, hipStream_t s);
}  // namespace gw
