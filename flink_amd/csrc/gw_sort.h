#pragma once
#include "gw_device.h"

namespace gw {
// Stable LSD radix sort of (key, uint32 value) pairs by key bits [lo, hi) (gw_sort.hip): digits of
// <= 9 bits, one launch per digit.  The result is in (k1, v1) if *result_in_alt, else in
// (k0, v0); v0 / v1 may be null (keys only).  iota: v0's contents are not read, the values are the
// arrival indices 0..n-1.  scratch: sort_scratch_bytes(n) bytes.
// n <= kSortMaxRecords: a tile's per-digit prefix is a 30-bit field of its look-back status
// word (two flag bits above it); a larger n returns hipErrorInvalidValue before any launch,
// and the callers split their batches below it.
constexpr int64_t kSortMaxRecords = ((int64_t)1 << 30) - 1;
int64_t sort_scratch_bytes(int64_t n);
hipError_t sort_pairs_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, int64_t n, int lo, int hi,
                          void* scratch, hipStream_t s, int* result_in_alt, bool iota = false);
hipError_t sort_pairs_u64(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, int64_t n, int lo, int hi,
                          void* scratch, hipStream_t s, int* result_in_alt, bool iota = false);
// sort_pairs_u64 over bits [0, bits) (the re-fire list)
int64_t radix_sort_scratch_bytes(int64_t n);
hipError_t radix_sort_pairs(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, int64_t n, int bits,
                            void* scratch, hipStream_t s, int* result_in_alt);
hipError_t launch_iota(uint32_t* v, int64_t n, hipStream_t s);
}  // namespace gw
