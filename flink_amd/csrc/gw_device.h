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
// Hot counters are sharded (blockIdx % kShards) and updated once per block after a
// wave + LDS reduction: same-address device atomics serialise at ~12 ns each on
// MI355X (MI355X_MICROARCH.md "fanin"), so one counter per wave costs ms per launch.
constexpr int kShards = 32;
struct ShardCtr {
    unsigned long long late, ins, flags, occ, cells, merges, pad0, pad1;  // 64 B
};
struct DevStatus {
    unsigned long long used_slots;  // host view: sum of sh[].ins
    unsigned long long n_deferred;  // deferred-list cursor (rare writers)
    unsigned long long late;        // host view: sum of sh[].late
    unsigned long long flags;       // host view: OR of sh[].flags
    unsigned long long occ;         // host view: OR of sh[].occ (pane-ring positions with data)
    unsigned long long rows;        // output cursor (one atomic per block flush)
    long long def_min_pane;         // min pane over the deferred list (reduction)
    unsigned long long preagg_cells;// host view: sum of sh[].cells
    unsigned long long merges;      // host view: sum of sh[].merges (session merges, M_b)
    unsigned long long overflow;    // session segments that did not fit (retry list length)
    unsigned long long spills;      // region apply: records left in the buffer by full regions
    unsigned long long n_refire;    // lateness > 0: re-fire list cursor (late records of fired windows)
    unsigned long long n_late_out;  // late side output cursor (GW_FLAG_LATE_SIDE_OUTPUT)
    unsigned long long wide_vals;   // compact region records: values beyond 32 bits sent to the deferred list
    unsigned long long fire_skip;   // k_fire_guard: 1 = the fire enqueued behind it does nothing
    unsigned long long fire_rows0;  // k_fire_guard: the output cursor before that fire
    unsigned long long pad[4];      // pad[kPubSeqWord]: stamp of a published host copy (never set on the device)
    ShardCtr sh[kShards];
};
constexpr int kPubSeqWord = 3;
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

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ unsigned long long wave_ior(unsigned long long v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}

// Block-level reduction of the per-thread counters, then ONE atomic per non-zero
// field into this block's shard.  Every thread of the block must call it (uniformly).
__device__ __forceinline__ void block_commit(DevStatus* st, unsigned long long late, unsigned long long ins,
                                             unsigned long long flags, unsigned long long occ,
                                             unsigned long long cells = 0, unsigned long long merges = 0) {
    __shared__ unsigned long long red[16][6];
    late = wave_sum(late); ins = wave_sum(ins); cells = wave_sum(cells); merges = wave_sum(merges);
    flags = wave_ior(flags); occ = wave_ior(occ);
    const int wave = threadIdx.x >> 6;
    if (__lane_id() == 0) {
        red[wave][0] = late; red[wave][1] = ins; red[wave][2] = flags;
        red[wave][3] = occ; red[wave][4] = cells; red[wave][5] = merges;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nw = (blockDim.x + 63) >> 6;
        unsigned long long v[6] = {0, 0, 0, 0, 0, 0};
        for (int w = 0; w < nw; ++w) {
            v[0] += red[w][0]; v[1] += red[w][1]; v[2] |= red[w][2];
            v[3] |= red[w][3]; v[4] += red[w][4]; v[5] += red[w][5];
        }
        ShardCtr& sc = st->sh[blockIdx.x % kShards];
        if (v[0]) atomicAdd(&sc.late, v[0]);
        if (v[1]) atomicAdd(&sc.ins, v[1]);
        if (v[2]) atomicOr(&sc.flags, v[2]);
        if (v[3]) atomicOr(&sc.occ, v[3]);
        if (v[4]) atomicAdd(&sc.cells, v[4]);
        if (v[5]) atomicAdd(&sc.merges, v[5]);
    }
}

// Fold the shards into the scalar host-view fields (host side, after a D2H copy).
inline void fold_shards(DevStatus* h) {
    unsigned long long late = 0, ins = 0, flags = 0, occ = 0, cells = 0, merges = 0;
    for (int i = 0; i < kShards; ++i) {
        late += h->sh[i].late; ins += h->sh[i].ins; flags |= h->sh[i].flags;
        occ |= h->sh[i].occ; cells += h->sh[i].cells; merges += h->sh[i].merges;
    }
    h->late = late; h->used_slots = ins; h->flags = flags; h->occ = occ;
    h->preagg_cells = cells; h->merges = merges;
}

// Fired-row staging in LDS: rows are appended with LDS atomics and flushed to the
// global output with one device atomic per flush and coalesced stores.
#ifndef GW_ROW_STAGE
#define GW_ROW_STAGE 1024
#endif
constexpr int kRowStage = GW_ROW_STAGE;  // rows a fire workgroup stages in LDS before one output reservation
struct RowStage {
    long long k[kRowStage], s[kRowStage], e[kRowStage], r[kRowStage];
    unsigned cnt;
    unsigned long long base;
};
__device__ __forceinline__ void stage_flush(RowStage& rs, unsigned long long* cursor, int64_t* ok, int64_t* os,
                                            int64_t* oe, int64_t* orr) {
    __syncthreads();
    const unsigned c = rs.cnt;
    if (threadIdx.x == 0 && c) rs.base = atomicAdd(cursor, (unsigned long long)c);
    __syncthreads();
    const unsigned long long b = rs.base;
    for (unsigned j = threadIdx.x; j < c; j += blockDim.x) {
        ok[b + j] = rs.k[j]; os[b + j] = rs.s[j]; oe[b + j] = rs.e[j]; orr[b + j] = rs.r[j];
    }
    __syncthreads();
    if (threadIdx.x == 0) rs.cnt = 0;
    __syncthreads();
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
        // a plain (cached) load: a key word only ever goes from kEmptyKey to a key, so a stale
        // read can only be kEmptyKey, which the CAS resolves (a volatile load here is a
        // system-scope sc0 sc1 load that skips the caches on every probe)
        const int64_t k = s[0];
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
