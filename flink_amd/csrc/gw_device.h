// gw_device.h — device-side data structures shared by the pane and session kernels.
//
// HBM state table: `cap` (power of two) slots + 1 sentinel slot for
// the key Long.MIN_VALUE (which doubles as the empty marker).  Slot layout, in
// int64 words:
//     [0] key            (kEmptyKey while free; set once by CAS)
//     [1] presence mask  (pane mode: bit r = ring cell r non-null;
//                         session mode: number of in-flight sessions)
//     [2 ...]            accumulator cells (pane mode) / sessions (session mode)
// The stride is a multiple of 64 B so a slot never straddles more 128-B L2 lines
// than necessary, and one probe + RMW touches one line for the common 64-B slot.
#pragma once
#include "gw_common.h"

namespace gw {

struct TableView {
    int64_t* base;    // cap+1 slots
    int64_t cap;      // power of two
    int32_t stride_w; // slot stride in int64 words
    int32_t ring;     // pane ring length R (pane mode) / sessions per slot K (session mode)
    int32_t words;    // int64 words per cell
    int32_t agg;
};

// Device-side counters, copied to pinned host memory after each launch sequence.
struct DevStatus {
    unsigned long long used_slots;
    unsigned long long n_deferred;
    unsigned long long late;
    unsigned long long flags;      // GW_DF_*
    unsigned long long occ;        // pane-ring positions that may hold data
    unsigned long long rows;       // output cursor
    long long def_min_pane;        // min pane over the deferred list (reduction)
    unsigned long long preagg_cells;
    unsigned long long merges;     // session merges (M_b)
    unsigned long long overflow;   // session slots that did not fit (retry list length)
    unsigned long long pad[6];
};
#define GW_DF_NO_TS 1ull
#define GW_DF_RANGE 2ull
#define GW_DF_TABLE_FULL 4ull

__device__ __forceinline__ int64_t* slot_ptr(const TableView& t, int64_t idx) {
    return t.base + idx * (int64_t)t.stride_w;
}

// Wave-aggregated atomic add of a per-lane count; returns this lane's exclusive
// offset into the reserved range (only meaningful when want_offset).
__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* ctr, bool pred) {
    const unsigned long long ballot = __ballot(pred);
    if (ballot == 0) return 0;
    const int lane = __lane_id();
    const int leader = __ffsll((long long)ballot) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(ballot));
    base = __shfl(base, leader);
    const unsigned long long below = ballot & ((1ull << lane) - 1ull);
    return base + (unsigned long long)__popcll(below);
}

__device__ __forceinline__ void wave_add(unsigned long long* ctr, unsigned long long v) {
    // v may differ per lane: reduce over the wave with DPP-backed shuffles
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (__lane_id() == 0 && v) atomicAdd(ctr, v);
}

__device__ __forceinline__ void wave_or(unsigned long long* ctr, unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    if (__lane_id() == 0 && v) atomicOr(ctr, v);
}

// Exclusive wave scan of per-lane counts + one atomic per wave.
__device__ __forceinline__ unsigned long long wave_reserve_n(unsigned long long* ctr, unsigned cnt) {
    const int lane = __lane_id();
    unsigned incl = cnt;
    for (int o = 1; o < 64; o <<= 1) {
        unsigned up = __shfl_up(incl, o);
        if (lane >= o) incl += up;
    }
    const unsigned total = __shfl(incl, 63);
    unsigned long long base = 0;
    if (lane == 63 && total) base = atomicAdd(ctr, (unsigned long long)total);
    base = __shfl(base, 63);
    return base + (incl - cnt);
}

// Find the slot of `key`, inserting it if absent (CAS on the key word).  Returns the
// slot index or -1 if the probe limit was hit.  `inserted` reports a new key.
__device__ __forceinline__ int64_t find_or_insert(const TableView& t, int64_t key, bool& inserted) {
    inserted = false;
    if (key == kEmptyKey) return t.cap;  // sentinel slot
    const uint64_t mask = (uint64_t)t.cap - 1;
    uint64_t idx = slot_hash(key) & mask;
    for (int p = 0; p < kMaxProbe; ++p) {
        int64_t* s = slot_ptr(t, (int64_t)idx);
        int64_t k = *(volatile int64_t*)s;  // a stale kEmptyKey is resolved by the CAS
        if (k == key) return (int64_t)idx;
        if (k == kEmptyKey) {
            unsigned long long prev = atomicCAS((unsigned long long*)s, (unsigned long long)kEmptyKey,
                                                (unsigned long long)key);
            if (prev == (unsigned long long)kEmptyKey) { inserted = true; return (int64_t)idx; }
            if ((int64_t)prev == key) return (int64_t)idx;
        }
        idx = (idx + 1) & mask;
    }
    return -1;
}

// Lookup without insert (rehash / snapshot).
__device__ __forceinline__ int64_t find_slot(const TableView& t, int64_t key) {
    if (key == kEmptyKey) return t.cap;
    const uint64_t mask = (uint64_t)t.cap - 1;
    uint64_t idx = slot_hash(key) & mask;
    for (int p = 0; p < kMaxProbe; ++p) {
        int64_t k = slot_ptr(t, (int64_t)idx)[0];
        if (k == key) return (int64_t)idx;
        if (k == kEmptyKey) return -1;
        idx = (idx + 1) & mask;
    }
    return -1;
}

// Atomic merge of one cell contribution (a0, a1) into cell `c` (device scope).
template <int AGG>
__device__ __forceinline__ void cell_atomic(int64_t* c, int64_t a0, int64_t a1) {
    if constexpr (AGG == GW_COUNT || AGG == GW_SUM_I64 || AGG == GW_SUM_I32) {
        atomicAdd((unsigned long long*)c, (unsigned long long)a0);
    } else if constexpr (AGG == GW_SUM_F64) {
        unsafeAtomicAdd((double*)c, bits_to_f64(a0));
    } else if constexpr (AGG == GW_MIN_I64 || AGG == GW_MIN_F64) {
        atomicMin((long long*)c, (long long)a0);
    } else if constexpr (AGG == GW_MAX_I64 || AGG == GW_MAX_F64) {
        atomicMax((long long*)c, (long long)a0);
    } else if constexpr (AGG == GW_AVG_I64) {
        atomicAdd((unsigned long long*)c, (unsigned long long)a0);
        atomicAdd((unsigned long long*)(c + 1), (unsigned long long)a1);
    } else {  // GW_AVG_F64
        unsafeAtomicAdd((double*)c, bits_to_f64(a0));
        atomicAdd((unsigned long long*)(c + 1), (unsigned long long)a1);
    }
}

template <int AGG>
__device__ __forceinline__ void fold_reg(int64_t& a0, int64_t& a1, int64_t b0, int64_t b1) {
    fold_cell(AGG, a0, a1, b0, b1);
}

}  // namespace gw
