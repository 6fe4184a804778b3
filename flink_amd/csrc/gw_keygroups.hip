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
// scatter (wave64 ballot matching for in-wave ranks, the tile ranked in LDS before any store).
#include "gw_kernels.h"

#include <algorithm>

namespace gw {

constexpr int kPartMaxDest = 256;
constexpr int kPartItems = 8;  // records per thread per block tile

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

// Bits that tell destinations 0..nd-1 apart: wave peer matching needs only these ballots
// (one at a single owner with packing, four at eight owners), not eight.
__host__ __device__ inline int dest_bits(int32_t nd) {
    int b = 0;
    while ((1 << b) < nd) ++b;
    return b;
}

// Lanes of this wave with destination d (valid lanes only).
__device__ __forceinline__ unsigned long long wave_peers(bool valid, int32_t d, int nbits) {
    unsigned long long peers = __ballot(valid);
    for (int b = 0; b < nbits; ++b) {
        const bool bit = (d >> b) & 1;
        const unsigned long long bb = __ballot(bit);
        peers &= bit ? bb : ~bb;
    }
    return peers;
}

// Destination bucket of one record from its loaded columns: its owner, or (packing)
// 2 * owner + (does not fit).
__device__ __forceinline__ int32_t dest_rec(int64_t k, int32_t kh, bool has_hash, int64_t t, bool has_val, int64_t v,
                                            int32_t max_p, int32_t p, const PackGeom& g, uint64_t& w) {
    const int32_t h = has_hash ? kh : java_long_hash(k);
    const int32_t o = operator_for_key_group(max_p, p, key_group_for_hash(h, max_p));
    if (!g.enabled) return o;
    return 2 * o + (pack_word(g, k, t, has_val, has_val ? v : 0, w) ? 0 : 1);
}

// pass 1: counts[block][dest].  The tile's columns are loaded before any counting (all loads
// in flight at once), and each wave adds its peers' count once per destination instead of one
// LDS atomic per record (one owner: every record of a wave hits the same counter).
__global__ void __launch_bounds__(256) k_part_hist(int64_t n, const int64_t* key, const int32_t* key_hash,
                                                   const int64_t* ts, const int64_t* val, int32_t max_p, int32_t p,
                                                   PackGeom g, uint32_t* block_counts) {
    __shared__ uint32_t h[kPartMaxDest];
    const int32_t nd = g.enabled ? 2 * p : p;
    const int nbits = dest_bits(nd);
    for (int d = threadIdx.x; d < nd; d += blockDim.x) h[d] = 0;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x * kPartItems + threadIdx.x;
    const bool has_hash = key_hash != nullptr, has_val = val != nullptr;
    int64_t kk[kPartItems], tt[kPartItems], vv[kPartItems];
    int32_t hh[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = t0 + (int64_t)it * blockDim.x;
        const bool ok = i < n;
        kk[it] = ok && !has_hash ? key[i] : 0;
        hh[it] = ok && has_hash ? key_hash[i] : 0;
        tt[it] = ok && g.enabled ? ts[i] : 0;
        vv[it] = ok && g.enabled && has_val ? val[i] : 0;
    }
    __syncthreads();
    const int lane = __lane_id();
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = t0 + (int64_t)it * blockDim.x;
        const bool ok = i < n;
        uint64_t w;
        const int32_t d = ok ? dest_rec(kk[it], hh[it], has_hash, tt[it], has_val, vv[it], max_p, p, g, w) : 0;
        const unsigned long long peers = wave_peers(ok, d, nbits);
        if (ok && __popcll(peers & ((1ull << lane) - 1ull)) == 0) atomicAdd(&h[d], (uint32_t)__popcll(peers));
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
// (key_out | ts_out | val_out), at positions of one shared numbering.  The whole tile is
// loaded and ranked before any store: per (item, wave, destination) the wave's peer count goes
// to LDS, one thread per destination turns the counts into tile-relative offsets in (item,
// wave) order -- which keeps the partition stable -- and every record is stored at its
// block offset + that offset + its rank among its wave's peers: two barriers per tile rather
// than three per item.  Dynamic LDS: kPartItems * 4 * nd counts + nd block offsets.
__global__ void __launch_bounds__(256) k_part_scatter(int64_t n, const int64_t* key, const int32_t* key_hash,
                                                      const int64_t* ts, const int64_t* val, int32_t max_p,
                                                      int32_t p_owners, PackGeom g, const int64_t* offsets,
                                                      int64_t* key_out, int64_t* ts_out, int64_t* val_out,
                                                      int32_t* hash_out, uint64_t* packed_out) {
    extern __shared__ int64_t part_lds[];
    const int32_t nd = g.enabled ? 2 * p_owners : p_owners;  // buckets
    int64_t* base = part_lds;                                 // [nd]
    uint32_t* cnt = (uint32_t*)(part_lds + nd);               // [kPartItems][4][nd]
    const int lane = __lane_id();
    const int wave = threadIdx.x >> 6;
    const int nbits = dest_bits(nd);
    for (int d = threadIdx.x; d < nd; d += blockDim.x) base[d] = offsets[(int64_t)d * gridDim.x + blockIdx.x];
    for (int e = threadIdx.x; e < kPartItems * 4 * nd; e += blockDim.x) cnt[e] = 0;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x * kPartItems + threadIdx.x;
    const bool has_hash = key_hash != nullptr, has_val = val != nullptr;
    int64_t kk[kPartItems], tt[kPartItems], vv[kPartItems];
    int32_t hh[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = t0 + (int64_t)it * blockDim.x;
        const bool ok = i < n;
        kk[it] = ok ? key[i] : 0;
        tt[it] = ok ? ts[i] : 0;
        vv[it] = ok && has_val ? val[i] : 0;
        hh[it] = ok && has_hash ? key_hash[i] : 0;
    }
    __syncthreads();  // base / cnt initialised
    int32_t dd[kPartItems];
    uint32_t rk[kPartItems];
    uint64_t ww[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = t0 + (int64_t)it * blockDim.x;
        const bool ok = i < n;
        ww[it] = 0;
        dd[it] = ok ? dest_rec(kk[it], hh[it], has_hash, tt[it], has_val, vv[it], max_p, p_owners, g, ww[it]) : -1;
        const unsigned long long peers = wave_peers(ok, dd[it], nbits);
        rk[it] = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (ok && rk[it] == 0) cnt[(it * 4 + wave) * nd + dd[it]] = (uint32_t)__popcll(peers);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nd; d += blockDim.x) {
        uint32_t run = 0;
        for (int e = 0; e < kPartItems * 4; ++e) {
            const uint32_t c = cnt[e * nd + d];
            cnt[e * nd + d] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int32_t d = dd[it];
        if (d < 0) continue;
        const int64_t pos = base[d] + cnt[(it * 4 + wave) * nd + d] + rk[it];
        if (g.enabled && !(d & 1)) {
            packed_out[pos] = ww[it];
        } else {
            key_out[pos] = kk[it];
            ts_out[pos] = tt[it];
            if (has_val) val_out[pos] = vv[it];
            if (hash_out) hash_out[pos] = hh[it];
        }
    }
}

// Single-pass partition into per-destination regions (the exchange's own layout; the
// contiguous gw_partition_device layout keeps the three passes above).  Destination q's
// records go to region q of capacity cap: packed words at packed_out + q * cap, other records
// at key_out / ts_out / val_out / hash_out + q * cap.  With a region per destination a record's
// position needs only the counts of the same destination in earlier tiles, so the histogram
// and scan passes go: tiles are taken in order from a counter (tile_ctr), each publishes its
// per-destination count and looks back over earlier tiles' published counts (decoupled
// look-back, as the grouping sort's passes do, gw_sort.hip), and the last tile writes the
// totals.  status: [ntiles][nd] words, zeroed before the launch.  Costs P * cap records of
// memory per buffer -- the exchange uses it up to kPartRegionMaxOwners owners.
// unstable: no look-back -- each tile takes its place in a region with one device atomic on
// that region's total in counts[] (zeroed before the launch), so tiles land in the order they
// get there and a region's records are not in arrival order.  The exchange uses it only for
// packed batches, whose handles (integer sums, counts, min, max) do not see per-key arrival
// order (the packed words already arrive behind the other records); the look-back walked
// hundreds of earlier tiles while a whole grid of tiles published at once (round 6: 130 us per
// 10M records alone, profiles/r6/exchange/unstable/).

constexpr uint64_t kPrLocal = 1ull << 62, kPrIncl = 1ull << 63, kPrMask = kPrLocal - 1;

__device__ __forceinline__ uint64_t part_look_back(const uint64_t* status, int64_t t, int nd, int d) {
    uint64_t excl = 0;
    for (int64_t q = t - 1;; q -= 4) {  // four earlier tiles' words per round trip
        uint64_t x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            x[j] = q - j >= 0 ? __hip_atomic_load(status + (q - j) * nd + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : kPrIncl;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            while (!(x[j] & (kPrLocal | kPrIncl)))
                x[j] = __hip_atomic_load(status + (q - j) * nd + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            excl += x[j] & kPrMask;
            if (x[j] & kPrIncl) return excl;
        }
    }
}

__global__ void __launch_bounds__(256) k_part_regions(int64_t n, const int64_t* key, const int32_t* key_hash,
                                                      const int64_t* ts, const int64_t* val, int32_t max_p,
                                                      int32_t p_owners, PackGeom g, int64_t cap, uint64_t* status,
                                                      uint32_t* tile_ctr, int64_t ntiles, int64_t* key_out,
                                                      int64_t* ts_out, int64_t* val_out, int32_t* hash_out,
                                                      uint64_t* packed_out, int64_t* counts, uint64_t* zero_next,
                                                      int64_t zero_words, int unstable) {
    extern __shared__ int64_t part_lds[];
    __shared__ int64_t s_tile;
    const int32_t nd = g.enabled ? 2 * p_owners : p_owners;
    int64_t* base = part_lds;                    // [nd]
    uint32_t* cnt = (uint32_t*)(part_lds + nd);  // [kPartItems][4][nd]
    const int lane = __lane_id();
    const int wave = threadIdx.x >> 6;
    const int nbits = dest_bits(nd);
    if (threadIdx.x == 0) s_tile = (int64_t)atomicAdd(tile_ctr, 1u);
    for (int e = threadIdx.x; e < kPartItems * 4 * nd; e += blockDim.x) cnt[e] = 0;
    // the other status half (the previous launch's, done): zeroed here for the next launch
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < zero_words;
         e += (int64_t)gridDim.x * blockDim.x)
        zero_next[e] = 0;
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t t0 = tile * blockDim.x * kPartItems + threadIdx.x;
    const bool has_hash = key_hash != nullptr, has_val = val != nullptr;
    int64_t kk[kPartItems], tt[kPartItems], vv[kPartItems];
    int32_t hh[kPartItems], dd[kPartItems];
    uint32_t rk[kPartItems];
    uint64_t ww[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = t0 + (int64_t)it * blockDim.x;
        const bool ok = i < n;
        kk[it] = ok ? key[i] : 0;
        tt[it] = ok ? ts[i] : 0;
        vv[it] = ok && has_val ? val[i] : 0;
        hh[it] = ok && has_hash ? key_hash[i] : 0;
    }
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = t0 + (int64_t)it * blockDim.x;
        const bool ok = i < n;
        ww[it] = 0;
        dd[it] = ok ? dest_rec(kk[it], hh[it], has_hash, tt[it], has_val, vv[it], max_p, p_owners, g, ww[it]) : -1;
        const unsigned long long peers = wave_peers(ok, dd[it], nbits);
        rk[it] = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (ok && rk[it] == 0) cnt[(it * 4 + wave) * nd + dd[it]] = (uint32_t)__popcll(peers);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nd; d += blockDim.x) {
        uint32_t run = 0;
        for (int e = 0; e < kPartItems * 4; ++e) {
            const uint32_t c = cnt[e * nd + d];
            cnt[e * nd + d] = run;
            run += c;
        }
        if (unstable) {  // a tile's place in each region by one device atomic on the region's total
            base[d] = run ? (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(counts) + d,
                                               (unsigned long long)run)
                          : 0;
            continue;
        }
        uint64_t* st = status + tile * nd + d;
        uint64_t excl = 0;
        if (tile == 0) {
            __hip_atomic_store(st, (uint64_t)run | kPrIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(st, (uint64_t)run | kPrLocal, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            excl = part_look_back(status, tile, nd, d);
            __hip_atomic_store(st, (excl + run) | kPrIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        base[d] = (int64_t)excl;
        if (tile == ntiles - 1) counts[d] = (int64_t)(excl + run);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int32_t d = dd[it];
        if (d < 0) continue;
        const int32_t q = g.enabled ? d >> 1 : d;
        const int64_t pos = q * cap + base[d] + cnt[(it * 4 + wave) * nd + d] + rk[it];
        if (g.enabled && !(d & 1)) {
            packed_out[pos] = ww[it];
        } else {
            key_out[pos] = kk[it];
            ts_out[pos] = tt[it];
            if (has_val) val_out[pos] = vv[it];
            if (hash_out) hash_out[pos] = hh[it];
        }
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

// counts are zeroed once read: the unstable region partition of the next batch on this set
// adds into them (each thread zeroes only the entries it read).
__global__ void __launch_bounds__(256) k_exchange_message(int64_t* counts, int32_t p, int64_t wm, int64_t cols,
                                                          int packed, int64_t* msg) {
    for (int q = threadIdx.x; q < p; q += blockDim.x) {
        const int64_t pk = packed ? counts[2 * q] : 0;
        msg[4 * q] = packed ? pk + counts[2 * q + 1] : counts[q];
        msg[4 * q + 1] = wm;
        msg[4 * q + 2] = cols;
        msg[4 * q + 3] = pk;
        if (packed) {
            counts[2 * q] = 0;
            counts[2 * q + 1] = 0;
        } else {
            counts[q] = 0;
        }
    }
}

hipError_t launch_exchange_message(int64_t* counts, int32_t p, int64_t wm, int64_t cols, int packed,
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
    const size_t lds = (size_t)nd * 8 + (size_t)kPartItems * 4 * nd * 4;
    hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)nb), dim3(256), lds, s, n, key, key_hash, ts, val, max_p, p, g,
                       off, key_out, ts_out, val_out, key_hash ? hash_out : nullptr, packed_out);
    return hipGetLastError();
}

int64_t partition_regions_scratch_bytes(int64_t cap, int32_t nd) {
    return 2 * (part_blocks(std::max<int64_t>(cap, 1)) * nd + 8) * 8;
}

hipError_t launch_partition_regions(int64_t n, const int64_t* key, const int32_t* key_hash, const int64_t* ts,
                                    const int64_t* val, int32_t max_p, int32_t p, int64_t cap, int64_t* key_out,
                                    int64_t* ts_out, int64_t* val_out, int32_t* hash_out, const PackGeom* pack,
                                    uint64_t* packed_out, int64_t* counts, void* scratch, hipStream_t s, int turn,
                                    int32_t nd_max, int unstable) {
    PackGeom g{};
    if (pack && pack->enabled) {
        if (key_hash || !packed_out || pack->pane <= 0) return hipErrorInvalidValue;
        g = *pack;
    }
    const int32_t nd = g.enabled ? 2 * p : p;
    if (p < 1 || p > kPartRegionMaxOwners || n > cap || n < 1 || (turn >= 0 && nd > nd_max))
        return hipErrorInvalidValue;
    const int64_t nb = part_blocks(n);
    uint64_t *status, *zero_next = nullptr;
    int64_t zero_words = 0;
    if (turn < 0) {  // stateless: zero this launch's words first
        status = (uint64_t*)scratch;
        hipError_t e = hipMemsetAsync(scratch, 0, (size_t)(nb * nd + 1) * 8, s);
        if (e != hipSuccess) return e;
    } else {  // two halves sized for cap: this launch's (zeroed by the last) and the next's
        const int64_t half = part_blocks(cap) * nd_max + 8;
        status = (uint64_t*)scratch + (turn & 1) * half;
        zero_next = (uint64_t*)scratch + ((turn + 1) & 1) * half;
        zero_words = half;
    }
    uint32_t* ctr = (uint32_t*)(status + nb * nd);
    const size_t lds = (size_t)nd * 8 + (size_t)kPartItems * 4 * nd * 4;
    hipLaunchKernelGGL(k_part_regions, dim3((unsigned)nb), dim3(256), lds, s, n, key, key_hash, ts, val, max_p, p,
                       g, cap, status, ctr, nb, key_out, ts_out, val_out, key_hash ? hash_out : nullptr, packed_out,
                       counts, zero_next, zero_words, unstable);
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
