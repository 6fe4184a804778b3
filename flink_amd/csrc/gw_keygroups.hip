// gw_keygroups.hip — key-group hashing and the keyBy partition on the device.
//
//   KeyGroupRangeAssignment.assignToKeyGroup / computeOperatorIndexForKeyGroup
//     (flink-runtime/src/main/java/org/apache/flink/runtime/state/
//      KeyGroupRangeAssignment.java:63-77,124-127) with MathUtils.murmurHash
//     (flink-core/src/main/java/org/apache/flink/util/MathUtils.java:137-155)
//   KeyGroupStreamPartitioner.selectChannel (flink-runtime/src/main/java/org/apache/
//     flink/streaming/runtime/partitioner/KeyGroupStreamPartitioner.java:55-64)
//
// The partition is a stable counting sort of the record columns by destination
// subtask (= GPU rank), the send-side half of the RCCL all-to-all that replaces the
// Netty keyBy shuffle.  Three passes: per-block histogram, one-block scan, stable
// scatter (wave64 ballot matching for in-wave ranks).
#include "gw_kernels.h"

namespace gw {

constexpr int kPartMaxDest = 256;
constexpr int kPartItems = 8;  // records per thread per block tile

__device__ __forceinline__ int32_t owner_of(const int64_t* key, const int32_t* key_hash, int64_t i,
                                            int32_t max_p, int32_t p) {
    const int32_t h = key_hash ? key_hash[i] : java_long_hash(key[i]);
    return operator_for_key_group(max_p, p, key_group_for_hash(h, max_p));
}

__global__ void __launch_bounds__(256) k_key_groups(int64_t n, const int64_t* key, const int32_t* key_hash,
                                                    int32_t max_p, int32_t p, int32_t* kg, int32_t* owner) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t h = key_hash ? key_hash[i] : java_long_hash(key[i]);
        const int32_t g = key_group_for_hash(h, max_p);
        if (kg) kg[i] = g;
        if (owner) owner[i] = operator_for_key_group(max_p, p, g);
    }
}

// Destination bucket of record i: its owner, or (packing) 2 * owner + (does not fit).
__device__ __forceinline__ int32_t dest_of(const int64_t* key, const int32_t* key_hash, const int64_t* ts,
                                           const int64_t* val, int64_t i, int32_t max_p, int32_t p,
                                           const PackGeom& g, uint64_t& w) {
    const int32_t o = owner_of(key, key_hash, i, max_p, p);
    if (!g.enabled) return o;
    return 2 * o + (pack_word(g, key[i], ts[i], val != nullptr, val ? val[i] : 0, w) ? 0 : 1);
}

// pass 1: counts[block][dest]
__global__ void __launch_bounds__(256) k_part_hist(int64_t n, const int64_t* key, const int32_t* key_hash,
                                                   const int64_t* ts, const int64_t* val, int32_t max_p, int32_t p,
                                                   PackGeom g, uint32_t* block_counts) {
    __shared__ uint32_t h[kPartMaxDest];
    const int32_t nd = g.enabled ? 2 * p : p;
    for (int d = threadIdx.x; d < nd; d += blockDim.x) h[d] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x * kPartItems;
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = t0 + (int64_t)it * blockDim.x + threadIdx.x;
        uint64_t w;
        if (i < n) atomicAdd(&h[dest_of(key, key_hash, ts, val, i, max_p, p, g, w)], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nd; d += blockDim.x) block_counts[(int64_t)d * gridDim.x + blockIdx.x] = h[d];
}

// pass 2: exclusive scan over (dest-major, block-minor); totals per dest.  One block: each
// thread sums a contiguous run of the counts, a wave-shuffle scan over the threads' sums, each
// thread writes its run's offsets; a destination's total is the difference of the offsets at
// its first entry and the next destination's (each found from its thread's prefix plus a walk
// of at most `per` counts) -- not a serial loop over the blocks per destination (that loop took
// ~320 us at 10M records: 4883 dependent loads per destination).
__global__ void __launch_bounds__(1024) k_part_scan(uint32_t* block_counts, int64_t nblk, int32_t p,
                                                    int64_t* offsets, int64_t* counts) {
    __shared__ unsigned long long part[1024];
    __shared__ unsigned long long wsum[16];
    const int64_t total = nblk * p;
    const int64_t per = (total + blockDim.x - 1) / blockDim.x;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int64_t lo = t * per, hi = min(total, lo + per);
    unsigned long long s = 0;
    for (int64_t i = lo; i < hi; ++i) s += block_counts[i];
    unsigned long long incl = s;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long up = __shfl_up(incl, o);
        if (lane >= o) incl += up;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    unsigned long long off = 0;
    for (int q = 0; q < w; ++q) off += wsum[q];
    const unsigned long long excl = off + incl - s;
    part[t] = excl;
    unsigned long long run = excl;
    for (int64_t i = lo; i < hi; ++i) { const unsigned long long v = block_counts[i]; offsets[i] = (int64_t)run; run += v; }
    __syncthreads();
    // offset of entry i (i <= total) from the thread prefixes
    auto offset_at = [&](int64_t i) -> unsigned long long {
        if (i >= total) {
            unsigned long long tot = 0;
            for (int q = 0; q < (int)(blockDim.x >> 6); ++q) tot += wsum[q];
            return tot;
        }
        const int64_t th = i / per;
        unsigned long long o = part[th];
        for (int64_t j = th * per; j < i; ++j) o += block_counts[j];
        return o;
    };
    for (int d = t; d < p; d += blockDim.x) counts[d] = (int64_t)(offset_at((int64_t)(d + 1) * nblk) - offset_at((int64_t)d * nblk));
}

// Packing: bucket 2q holds q's packed words (packed_out), bucket 2q + 1 its other records
// (key_out | ts_out | val_out), at positions of one shared numbering.
__global__ void __launch_bounds__(256) k_part_scatter(int64_t n, const int64_t* key, const int32_t* key_hash,
                                                      const int64_t* ts, const int64_t* val, int32_t max_p,
                                                      int32_t p_owners, PackGeom g, const int64_t* offsets,
                                                      int64_t* key_out, int64_t* ts_out, int64_t* val_out,
                                                      int32_t* hash_out, uint64_t* packed_out) {
    __shared__ int64_t cursor[kPartMaxDest];
    __shared__ uint32_t wave_cnt[4][kPartMaxDest];
    const int lane = __lane_id();
    const int wave = threadIdx.x >> 6;
    const int32_t p = g.enabled ? 2 * p_owners : p_owners;  // buckets
    for (int d = threadIdx.x; d < p; d += blockDim.x) cursor[d] = offsets[(int64_t)d * gridDim.x + blockIdx.x];
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x * kPartItems;
    for (int it = 0; it < kPartItems; ++it) {
        for (int d = threadIdx.x; d < 4 * p; d += blockDim.x) wave_cnt[d / p][d % p] = 0;
        __syncthreads();
        const int64_t i = t0 + (int64_t)it * blockDim.x + threadIdx.x;
        const bool valid = i < n;
        uint64_t w = 0;
        const int32_t d = valid ? dest_of(key, key_hash, ts, val, i, max_p, p_owners, g, w) : -1;
        // peers: lanes of this wave with the same destination (8 ballots cover p <= 256)
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1;
            const unsigned long long bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const unsigned rank_in_wave = (unsigned)__popcll(peers & ((1ull << lane) - 1ull));
        if (valid && rank_in_wave == 0) wave_cnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            int64_t pos = cursor[d] + rank_in_wave;
            for (int q = 0; q < wave; ++q) pos += wave_cnt[q][d];
            if (g.enabled && !(d & 1)) {
                packed_out[pos] = w;
            } else {
                key_out[pos] = key[i];
                ts_out[pos] = ts[i];
                if (val) val_out[pos] = val[i];
                if (hash_out) hash_out[pos] = key_hash[i];
            }
        }
        __syncthreads();
        for (int dd = threadIdx.x; dd < p; dd += blockDim.x)
            cursor[dd] += wave_cnt[0][dd] + wave_cnt[1][dd] + wave_cnt[2][dd] + wave_cnt[3][dd];
        __syncthreads();
    }
}

// Ingest-side key checks (gw_ingest* with a key_hash column, or GW_FLAG_CHECK_KEY_GROUPS):
//   out[0] |= 1 when a key_hash differs from Long.hashCode(key): the window state groups keys
//          by Long.hashCode (snapshots, rescaling), so such a handle refuses to snapshot;
//   out[1] = min over records of (key group + 1) outside [kg_lo, kg_hi] (0: none), which
//          fails the batch like StateTable.getMapForKeyGroup (RR/state/heap/StateTable.java:
//          325-333, KeyGroupRangeOffsets.newIllegalKeyGroupException).
__global__ void __launch_bounds__(256) k_check_keys(int64_t n, const int64_t* key, const int32_t* key_hash,
                                                    int32_t max_p, int32_t kg_lo, int32_t kg_hi, int check_range,
                                                    unsigned long long* out) {
    unsigned long long foreign = 0, bad = ~0ull;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t lh = java_long_hash(key[i]);
        const int32_t h = key_hash ? key_hash[i] : lh;
        foreign |= (unsigned long long)(h != lh);
        if (check_range) {
            const int32_t g = key_group_for_hash(h, max_p);
            if (g < kg_lo || g > kg_hi) bad = min(bad, (unsigned long long)g + 1);
        }
    }
    foreign = wave_ior(foreign);
    for (int o = 32; o > 0; o >>= 1) bad = min(bad, (unsigned long long)__shfl_xor(bad, o));
    if (__lane_id() == 0) {
        if (foreign) atomicOr(&out[0], 1ull);
        if (bad != ~0ull) atomicMin(&out[1], bad);
    }
}

hipError_t launch_check_keys(int64_t n, const int64_t* key, const int32_t* key_hash, int32_t max_p, int32_t kg_lo,
                             int32_t kg_hi, int check_range, unsigned long long* out, hipStream_t s) {
    int64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_check_keys, dim3((unsigned)g), dim3(256), 0, s, n, key, key_hash, max_p, kg_lo, kg_hi,
                       check_range, out);
    return hipGetLastError();
}

// ---- key -> Java hashCode map (KeyHashMap, gw_kernels.h) --------------------------------
__device__ __forceinline__ int64_t khm_slot(const KeyHashMap& m, int64_t k) {
    return (int64_t)(slot_hash(k) & (uint64_t)(m.cap - 1));
}

__global__ void __launch_bounds__(256) k_khmap_insert(KeyHashMap m, int64_t n, const int64_t* key, const int32_t* hash,
                                                      int verify, unsigned long long* out) {
    unsigned long long ins = 0, bad = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = key[i];
        const int32_t h = hash[i];
        if (k == kEmptyKey) {  // the sentinel key has the extra slot
            if (verify) bad += m.hash[m.cap] != h;
            else if (atomicCAS((unsigned long long*)&m.key[m.cap], 0ull, 1ull) == 0ull) { m.hash[m.cap] = h; ins++; }
            continue;
        }
        for (int64_t s = khm_slot(m, k);; s = (s + 1) & (m.cap - 1)) {
            const int64_t cur = m.key[s];
            if (cur == k) {
                if (verify) bad += m.hash[s] != h;
                break;
            }
            if (verify) {
                if (cur == kEmptyKey) { bad++; break; }  // (cannot happen after the insert pass)
                continue;
            }
            if (cur != kEmptyKey) continue;
            const unsigned long long prev =
                atomicCAS((unsigned long long*)&m.key[s], (unsigned long long)kEmptyKey, (unsigned long long)k);
            if (prev == (unsigned long long)kEmptyKey) {
                m.hash[s] = h;  // records of one key carry one hash: concurrent writers agree
                ins++;
                break;
            }
            if ((int64_t)prev == k) break;
        }
    }
    ins = wave_sum(ins);
    bad = wave_sum(bad);
    if (__lane_id() == 0) {
        if (ins) atomicAdd(&out[0], ins);
        if (bad) atomicAdd(&out[1], bad);
    }
}

__global__ void __launch_bounds__(256) k_khmap_rehash(KeyHashMap f, KeyHashMap t) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < f.cap; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = f.key[i];
        if (k == kEmptyKey) continue;
        for (int64_t s = khm_slot(t, k);; s = (s + 1) & (t.cap - 1)) {
            if (atomicCAS((unsigned long long*)&t.key[s], (unsigned long long)kEmptyKey, (unsigned long long)k) ==
                (unsigned long long)kEmptyKey) {
                t.hash[s] = f.hash[i];
                break;
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        t.key[t.cap] = f.key[f.cap];
        t.hash[t.cap] = f.hash[f.cap];
    }
}

__global__ void __launch_bounds__(256) k_fill64(int64_t* p, int64_t n, int64_t v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

hipError_t launch_fill64(int64_t* p, int64_t n, int64_t v, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_fill64, dim3((unsigned)g), dim3(256), 0, s, p, n, v);
    return hipGetLastError();
}

__global__ void __launch_bounds__(256) k_exchange_message(const int64_t* counts, int32_t p, int64_t wm, int64_t cols,
                                                          int packed, int64_t* msg) {
    for (int q = threadIdx.x; q < p; q += blockDim.x) {
        const int64_t pk = packed ? counts[2 * q] : 0;
        msg[4 * q] = packed ? pk + counts[2 * q + 1] : counts[q];
        msg[4 * q + 1] = wm;
        msg[4 * q + 2] = cols;
        msg[4 * q + 3] = pk;
    }
}

hipError_t launch_exchange_message(const int64_t* counts, int32_t p, int64_t wm, int64_t cols, int packed,
                                   int64_t* msg, hipStream_t s) {
    hipLaunchKernelGGL(k_exchange_message, dim3(1), dim3(256), 0, s, counts, p, wm, cols, packed, msg);
    return hipGetLastError();
}

hipError_t launch_khmap_insert(const KeyHashMap& m, int64_t n, const int64_t* key, const int32_t* hash, int verify,
                               unsigned long long* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_khmap_insert, dim3((unsigned)g), dim3(256), 0, s, m, n, key, hash, verify, out);
    return hipGetLastError();
}

hipError_t launch_khmap_rehash(const KeyHashMap& from, const KeyHashMap& to, hipStream_t s) {
    int64_t g = (from.cap + 255) / 256;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_khmap_rehash, dim3((unsigned)g), dim3(256), 0, s, from, to);
    return hipGetLastError();
}

hipError_t launch_key_groups(int64_t n, const int64_t* key, const int32_t* key_hash, int32_t max_p,
                             int32_t p, int32_t* kg, int32_t* owner, hipStream_t s) {
    int64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_key_groups, dim3((unsigned)g), dim3(256), 0, s, n, key, key_hash, max_p, p, kg, owner);
    return hipGetLastError();
}

static int64_t part_blocks(int64_t n) {
    int64_t b = (n + 256 * kPartItems - 1) / (256 * kPartItems);
    return b < 1 ? 1 : b;
}

int64_t partition_scratch_bytes(int64_t n, int32_t p) {
    const int64_t nb = part_blocks(n);
    return nb * p * (int64_t)sizeof(uint32_t) + nb * p * (int64_t)sizeof(int64_t) + 256;
}

hipError_t launch_partition(int64_t n, const int64_t* key, const int32_t* key_hash, const int64_t* ts,
                            const int64_t* val, int32_t max_p, int32_t p, int64_t* key_out, int64_t* ts_out,
                            int64_t* val_out, int64_t* counts, void* scratch, hipStream_t s, int32_t* hash_out,
                            const PackGeom* pack, uint64_t* packed_out) {
    PackGeom g{};
    if (pack && pack->enabled) {
        if (key_hash || !packed_out || pack->pane <= 0) return hipErrorInvalidValue;
        g = *pack;
    }
    const int32_t nd = g.enabled ? 2 * p : p;
    if (p < 1 || nd > kPartMaxDest) return hipErrorInvalidValue;
    const int64_t nb = part_blocks(n);
    uint32_t* bc = (uint32_t*)scratch;
    int64_t* off = (int64_t*)(((uintptr_t)(bc + nb * nd) + 15) & ~(uintptr_t)15);
    hipLaunchKernelGGL(k_part_hist, dim3((unsigned)nb), dim3(256), 0, s, n, key, key_hash, ts, val, max_p, p, g, bc);
    hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(1024), 0, s, bc, nb, nd, off, counts);
    hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)nb), dim3(256), 0, s, n, key, key_hash, ts, val, max_p, p, g,
                       off, key_out, ts_out, val_out, key_hash ? hash_out : nullptr, packed_out);
    return hipGetLastError();
}

// Packed words back to (key, ts, value): ts = the start of the word's pane.
__global__ void __launch_bounds__(256) k_unpack(int64_t n, const uint64_t* w, PackGeom g, int64_t* key, int64_t* ts,
                                                int64_t* val) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t k, t, v;
        unpack_word(g, w[i], k, t, v);
        key[i] = k;
        ts[i] = t;
        if (val) val[i] = v;
    }
}

hipError_t launch_unpack(int64_t n, const uint64_t* w, const PackGeom& g, int64_t* key, int64_t* ts, int64_t* val,
                         hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t b = (n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(k_unpack, dim3((unsigned)b), dim3(256), 0, s, n, w, g, key, ts, val);
    return hipGetLastError();
}

}  // namespace gw
