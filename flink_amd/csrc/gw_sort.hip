// gw_sort.hip — hand-written stable LSD radix sort of (key, uint32 value) pairs for gfx950,
// one kernel launch per digit ("onesweep": decoupled look-back instead of a histogram pass per
// digit and a device-wide scan).
//
// Used to group records by key in arrival order: the session path's (state slot, arrival)
// grouping -- the GPU analogue of MergingWindowSet replaying a key's elements in order
// (MergingWindowSet.addWindow, RS/runtime/operators/windowing/MergingWindowSet.java:153-224) --,
// the count-window path, the re-fire list (lateness > 0) and the first-element join.
//
// Per sort: one histogram kernel reads the keys once and counts every digit's bins; one block
// scans them.  Per digit (<= 9 bits, so 26-bit slots take 3 passes), a persistent grid takes
// 4096-record tiles in order; for each tile:
//   * the records load striped within a wave (coalesced), and each wave ranks its 1024 records
//     in order against wave-private digit counters: a wave multi-split (one ballot per digit
//     bit gives each lane the mask of lanes with its digit; the lowest of them bumps the counter
//     by the group's size) -- stable, and no LDS atomics;
//   * per digit, one thread publishes the tile's count, looks back over the preceding tiles'
//     published counts / inclusive prefixes (flag in the top two bits of one 32-bit word,
//     agent-scope loads and stores: the tiles run on different XCDs, whose L2s are not
//     coherent), and publishes the tile's inclusive prefix;
//   * the tile is reordered in LDS by digit and written out bin run by bin run (coalesced).
// Tiles are taken in blockIdx order by a grid no larger than what stays resident, so a tile's
// predecessors are always running or done: the look-back always terminates.
#include "gw_sort.h"

#include <algorithm>

namespace gw {

constexpr int kOsThreads = 256;
constexpr int kOsItems = 16;
constexpr int kOsTile = kOsThreads * kOsItems;  // 4096
constexpr int kOsWaves = kOsThreads / 64;
constexpr uint32_t kOsLocal = 1u << 30, kOsIncl = 2u << 30, kOsMask = (1u << 30) - 1;

struct SortPlan {
    int npass;
    int shift[8], width[8];
};

static SortPlan plan_for(int lo, int hi) {
    SortPlan p{};
    const int bits = std::max(0, hi - lo);
    p.npass = (bits + 8) / 9;  // digits of <= 9 bits
    if (p.npass > 8) p.npass = 8;
    int at = lo;
    for (int i = 0; i < p.npass; ++i) {
        const int w = (bits - (at - lo) + (p.npass - i) - 1) / (p.npass - i);  // spread the bits evenly
        p.shift[i] = at;
        p.width[i] = w;
        at += w;
    }
    return p;
}

template <typename K>
__device__ __forceinline__ uint32_t digit_of(K k, int shift, int width) {
    return (uint32_t)(k >> shift) & ((1u << width) - 1u);
}

// Counts of every digit's bins over all keys: ghist[pass][512].
template <typename K>
__global__ void __launch_bounds__(256) k_os_hist(const K* keys, int64_t n, SortPlan p, uint32_t* ghist) {
    __shared__ uint32_t h[8][512];
    for (int i = threadIdx.x; i < p.npass * 512; i += blockDim.x) h[i >> 9][i & 511] = 0;
    __syncthreads();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const K k = keys[i];
        for (int q = 0; q < p.npass; ++q) atomicAdd(&h[q][digit_of(k, p.shift[q], p.width[q])], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < p.npass * 512; i += blockDim.x) {
        const uint32_t v = h[i >> 9][i & 511];
        if (v) atomicAdd(&ghist[i], v);
    }
}

// Exclusive scan of each pass's 512 bins in place (one block of 512 threads).
__global__ void __launch_bounds__(512) k_os_scan(uint32_t* ghist, int npass) {
    __shared__ uint32_t wsum[8];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int q = 0; q < npass; ++q) {
        const uint32_t v = ghist[q * 512 + t];
        uint32_t incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t up = __shfl_up(incl, o);
            if (lane >= o) incl += up;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (int i = 0; i < w; ++i) off += wsum[i];
        ghist[q * 512 + t] = off + incl - v;
        __syncthreads();
    }
}

// One digit pass over n records: tiles t = blockIdx.x, blockIdx.x + gridDim.x, ...
template <typename K, bool V>
__global__ void __launch_bounds__(kOsThreads) k_os_pass(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                        K* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n,
                                                        int shift, int width, const uint32_t* __restrict__ gbase,
                                                        uint32_t* status, int64_t ntiles) {
    __shared__ uint32_t cnt[kOsWaves][512];  // per wave: running count of each digit; then its base
    __shared__ uint32_t lstart[513];         // the tile's exclusive scan over digits
    __shared__ uint32_t gstart[512];         // global position of the tile's first record of a digit
    __shared__ uint32_t wsum[kOsWaves];
    __shared__ K s_k[kOsTile];
    __shared__ uint32_t s_v[V ? kOsTile : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nbins = 1 << width;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t base = t * kOsTile;
        const int cnt_t = (int)min((int64_t)kOsTile, n - base);
        for (int i = threadIdx.x; i < kOsWaves * 512; i += kOsThreads) (&cnt[0][0])[i] = 0;
        K k[kOsItems];
        uint32_t v[kOsItems], d[kOsItems], r[kOsItems];
#pragma unroll
        for (int j = 0; j < kOsItems; ++j) {  // wave w: records [w * 1024, (w + 1) * 1024), striped
            const int e = wave * (64 * kOsItems) + j * 64 + lane;
            k[j] = e < cnt_t ? kin[base + e] : (K)0;
            if constexpr (V) v[j] = e < cnt_t ? vin[base + e] : 0u;
        }
        __syncthreads();  // the counters are zero
#pragma unroll
        for (int j = 0; j < kOsItems; ++j) {  // in order: stable within the wave
            const int e = wave * (64 * kOsItems) + j * 64 + lane;
            const bool valid = e < cnt_t;
            d[j] = digit_of(k[j], shift, width);
            uint64_t peers = __ballot(valid);
            for (int b = 0; b < width; ++b) {
                const bool bit = (d[j] >> b) & 1u;
                const uint64_t bb = __ballot(bit);
                peers &= bit ? bb : ~bb;
            }
            const uint32_t below = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
            uint32_t old = 0;
            if (valid && below == 0) {  // the group's lowest lane: only this wave writes its counters
                old = cnt[wave][d[j]];
                cnt[wave][d[j]] = old + (uint32_t)__popcll(peers);
            }
            old = __shfl(old, valid ? __ffsll((long long)peers) - 1 : lane);
            r[j] = old + below;
        }
        __syncthreads();
        // per digit: the waves' bases within the digit, the tile's count, its global position
        for (int b = threadIdx.x; b < nbins; b += kOsThreads) {
            uint32_t tot = 0;
#pragma unroll
            for (int w = 0; w < kOsWaves; ++w) {
                const uint32_t c = cnt[w][b];
                cnt[w][b] = tot;
                tot += c;
            }
            uint32_t* st = status + t * 512 + b;
            if (t == 0) {
                __hip_atomic_store(st, tot | kOsIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gstart[b] = gbase[b];
            } else {
                __hip_atomic_store(st, tot | kOsLocal, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                uint32_t excl = 0;
                for (int64_t q = t - 1; q >= 0; --q) {  // decoupled look-back
                    uint32_t x;
                    do {
                        x = __hip_atomic_load(status + q * 512 + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } while (!(x & (kOsLocal | kOsIncl)));
                    excl += x & kOsMask;
                    if (x & kOsIncl) break;
                }
                __hip_atomic_store(st, (excl + tot) | kOsIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gstart[b] = gbase[b] + excl;
            }
            lstart[b] = tot;  // scanned below
        }
        __syncthreads();
        {  // exclusive scan of the tile's digit counts (<= 512: two per thread)
            const int t2 = threadIdx.x;
            const uint32_t a0 = 2 * t2 < nbins ? lstart[2 * t2] : 0u, a1 = 2 * t2 + 1 < nbins ? lstart[2 * t2 + 1] : 0u;
            uint32_t incl = a0 + a1;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t up = __shfl_up(incl, o);
                if (lane >= o) incl += up;
            }
            if (lane == 63) wsum[wave] = incl;
            __syncthreads();
            uint32_t off = 0;
            for (int w = 0; w < wave; ++w) off += wsum[w];
            const uint32_t ex = off + incl - (a0 + a1);
            if (2 * t2 < nbins) lstart[2 * t2] = ex;
            if (2 * t2 + 1 < nbins) lstart[2 * t2 + 1] = ex + a0;
            if (t2 == kOsThreads - 1) lstart[nbins] = off + incl;
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < kOsItems; ++j) {  // reorder the tile by digit in LDS
            const int e = wave * (64 * kOsItems) + j * 64 + lane;
            if (e < cnt_t) {
                const uint32_t lp = lstart[d[j]] + cnt[wave][d[j]] + r[j];
                s_k[lp] = k[j];
                if constexpr (V) s_v[lp] = v[j];
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < cnt_t; i += kOsThreads) {  // out, bin run by bin run
            const K kk = s_k[i];
            const uint32_t dd = digit_of(kk, shift, width);
            const uint32_t at = gstart[dd] + (uint32_t)i - lstart[dd];
            kout[at] = kk;
            if constexpr (V) vout[at] = s_v[i];
        }
        __syncthreads();  // LDS reused by the next tile
    }
}

__global__ void __launch_bounds__(256) k_iota(uint32_t* v, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[i] = (uint32_t)i;
}

static int64_t os_tiles(int64_t n) { return n <= 0 ? 0 : (n + kOsTile - 1) / kOsTile; }

int64_t sort_scratch_bytes(int64_t n) { return (8 * 512 + os_tiles(std::max<int64_t>(n, 1)) * 512) * 4 + 256; }
int64_t radix_sort_scratch_bytes(int64_t n) { return sort_scratch_bytes(n); }

template <typename K, bool V>
static int grid_of_pass() {
    static int g = 0;
    if (!g) {
        int dev = 0, cus = 0, per = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k_os_pass<K, V>, kOsThreads, 0);
        g = std::max(1, cus) * std::max(1, per);
    }
    return g;
}

template <typename K>
static hipError_t sort_pairs_impl(K* k0, uint32_t* v0, K* k1, uint32_t* v1, int64_t n, int lo, int hi, void* scratch,
                                  hipStream_t s, int* result_in_alt) {
    *result_in_alt = 0;
    const SortPlan p = plan_for(lo, hi);
    if (n <= 1 || p.npass == 0) return hipSuccess;
    uint32_t* ghist = (uint32_t*)scratch;
    uint32_t* status = ghist + 8 * 512;
    const int64_t nt = os_tiles(n);
    hipError_t e = hipMemsetAsync(ghist, 0, (size_t)p.npass * 512 * 4, s);
    if (e != hipSuccess) return e;
    const int hg = (int)std::min<int64_t>(2048, (n + 255) / 256);
    hipLaunchKernelGGL(k_os_hist<K>, dim3(hg), dim3(256), 0, s, (const K*)k0, n, p, ghist);
    hipLaunchKernelGGL(k_os_scan, dim3(1), dim3(512), 0, s, ghist, p.npass);
    int alt = 0;
    for (int q = 0; q < p.npass; ++q) {
        K* kin = alt ? k1 : k0;
        K* kout = alt ? k0 : k1;
        uint32_t* vin = alt ? v1 : v0;
        uint32_t* vout = alt ? v0 : v1;
        if ((e = hipMemsetAsync(status, 0, (size_t)nt * 512 * 4, s)) != hipSuccess) return e;
        if (v0) {
            const int g = (int)std::min<int64_t>(nt, grid_of_pass<K, true>());
            hipLaunchKernelGGL((k_os_pass<K, true>), dim3(g), dim3(kOsThreads), 0, s, kin, vin, kout, vout, n,
                               p.shift[q], p.width[q], ghist + q * 512, status, nt);
        } else {
            const int g = (int)std::min<int64_t>(nt, grid_of_pass<K, false>());
            hipLaunchKernelGGL((k_os_pass<K, false>), dim3(g), dim3(kOsThreads), 0, s, kin, nullptr, kout, nullptr, n,
                               p.shift[q], p.width[q], ghist + q * 512, status, nt);
        }
        alt ^= 1;
    }
    *result_in_alt = alt;
    return hipGetLastError();
}

hipError_t sort_pairs_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, int64_t n, int lo, int hi,
                          void* scratch, hipStream_t s, int* result_in_alt) {
    return sort_pairs_impl<uint32_t>(k0, v0, k1, v1, n, lo, hi, scratch, s, result_in_alt);
}
hipError_t sort_pairs_u64(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, int64_t n, int lo, int hi,
                          void* scratch, hipStream_t s, int* result_in_alt) {
    return sort_pairs_impl<uint64_t>(k0, v0, k1, v1, n, lo, hi, scratch, s, result_in_alt);
}

hipError_t radix_sort_pairs(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, int64_t n, int bits,
                            void* scratch, hipStream_t s, int* result_in_alt) {
    return sort_pairs_u64(k0, v0, k1, v1, n, 0, bits, scratch, s, result_in_alt);
}

hipError_t launch_iota(uint32_t* v, int64_t n, hipStream_t s) {
    int64_t g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(k_iota, dim3((unsigned)g), dim3(256), 0, s, v, n);
    return hipGetLastError();
}

}  // namespace gw
