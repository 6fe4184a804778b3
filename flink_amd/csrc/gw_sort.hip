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
// scans them.  Per digit (<= 9 bits, so 26-bit slots take 3 passes), one workgroup per tile of
// NT x NI records, tiles numbered in the order the workgroups start (an atomic counter, so a
// tile's predecessors always run before it or beside it: the look-back cannot wait on a tile
// that is not yet resident, whatever else shares the GPU).  For each tile:
//   * the records load striped within a wave (coalesced), and each wave ranks its 64 NI records
//     in order against wave-private digit counters: a wave multi-split (one ballot per digit
//     bit gives each lane the mask of lanes with its digit; the lowest of them bumps the counter
//     by the group's size) -- stable, and no LDS atomics;
//   * per digit, one thread publishes the tile's count, looks back over the preceding tiles'
//     published counts / inclusive prefixes four tiles at a time (flag in the top two bits of
//     one 32-bit word, agent-scope loads and stores: the tiles run on different XCDs, whose L2s
//     are not coherent), and publishes the tile's inclusive prefix;
//   * the tile is reordered in LDS by digit and written out bin run by bin run (coalesced).
// The look-back words of the next pass are zeroed by the current one (one memset per sort).
#include "gw_sort.h"

#include <algorithm>
#include <cstdlib>

namespace gw {

constexpr uint32_t kOsLocal = 1u << 30, kOsIncl = 2u << 30, kOsMask = (1u << 30) - 1;
constexpr int kOsMaxBins = 512;
// Experiment builds only (flink_amd.build --define GW_SORT_EXP=n --out ...), results discarded:
// 1 no look-back, 2 no ranking, 4 no write-out.  The product library is built with 0.
#ifndef GW_SORT_EXP
#define GW_SORT_EXP 0
#endif

struct SortPlan {
    int npass;
    int shift[8], width[8];
};

static SortPlan plan_for(int lo, int hi, int maxw) {
    SortPlan p{};
    const int bits = std::max(0, hi - lo);
    p.npass = (bits + maxw - 1) / maxw;  // digits of <= maxw bits
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

// Counts of every digit's bins over all keys: ghist[pass][512].  A small grid (two blocks per
// CU) keeps the global atomics of the block totals few.  (A last-block-done scan here instead
// of k_os_scan measured 6x slower: the per-block release fence writes back the XCD's L2.)
template <typename K>
__global__ void __launch_bounds__(1024) k_os_hist(const K* keys, int64_t n, SortPlan p, uint32_t* ghist) {
    __shared__ uint32_t h[8][kOsMaxBins];
    for (int i = threadIdx.x; i < p.npass * kOsMaxBins; i += blockDim.x) h[i / kOsMaxBins][i % kOsMaxBins] = 0;
    __syncthreads();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const K k = keys[i];
        for (int q = 0; q < p.npass; ++q) atomicAdd(&h[q][digit_of(k, p.shift[q], p.width[q])], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < p.npass * kOsMaxBins; i += blockDim.x) {
        const uint32_t v = h[i / kOsMaxBins][i % kOsMaxBins];
        if (v) atomicAdd(&ghist[i], v);
    }
}

// Exclusive scan of each pass's 512 bins in place (one block of 512 threads).
__global__ void __launch_bounds__(512) k_os_scan(uint32_t* ghist, int npass) {
    __shared__ uint32_t wsum[8];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int q = 0; q < npass; ++q) {
        const uint32_t v = ghist[q * kOsMaxBins + t];
        uint32_t incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t up = __shfl_up(incl, o);
            if (lane >= o) incl += up;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (int i = 0; i < w; ++i) off += wsum[i];
        ghist[q * kOsMaxBins + t] = off + incl - v;
        __syncthreads();
    }
}

// Decoupled look-back of tile t for digit b: the sum of the preceding tiles' counts, read four
// tiles at a time (the loads of a group are issued together; a tile not yet published is
// re-read until it is).
__device__ __forceinline__ uint32_t os_look_back(const uint32_t* status, int64_t t, int b) {
    uint32_t excl = 0;
    for (int64_t q = t - 1;; q -= 4) {
        uint32_t x[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            x[j] = q - j >= 0 ? __hip_atomic_load(status + (q - j) * kOsMaxBins + b, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                              : kOsIncl;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            while (!(x[j] & (kOsLocal | kOsIncl)))
                x[j] = __hip_atomic_load(status + (q - j) * kOsMaxBins + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            excl += x[j] & kOsMask;
            if (x[j] & kOsIncl) return excl;
        }
    }
}

// One digit pass over n records: one tile of NT * NI records per workgroup.
template <typename K, bool V, int NT, int NI>
__global__ void __launch_bounds__(NT) k_os_pass(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                K* __restrict__ kout, uint32_t* __restrict__ vout, int64_t n,
                                                int shift, int width, const uint32_t* __restrict__ gbase,
                                                uint32_t* status, uint32_t* next_status, int64_t ntiles,
                                                uint32_t* tile_ctr) {
    constexpr int exp = GW_SORT_EXP;
    constexpr int NW = NT / 64, TILE = NT * NI;
    __shared__ uint32_t cnt[NW][kOsMaxBins];  // per wave: running count of each digit; then its base
    __shared__ uint32_t lstart[kOsMaxBins + 1];  // the tile's exclusive scan over digits
    __shared__ uint32_t gstart[kOsMaxBins];      // global position of the tile's first record of a digit
    __shared__ uint32_t wsum[NW];
    __shared__ K s_k[TILE];
    __shared__ uint32_t s_v[V ? TILE : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nbins = 1 << width;
    if (next_status)  // the next pass's look-back words (the pass before this one used them)
        for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < ntiles * kOsMaxBins; i += (int64_t)gridDim.x * NT)
            next_status[i] = 0;
    __shared__ uint32_t s_tile;
    if (threadIdx.x == 0) s_tile = atomicAdd(tile_ctr, 1u);  // tiles in order of the blocks' start
    __syncthreads();
    {
        const int64_t t = s_tile;
        const int64_t base = t * TILE;
        const int cnt_t = (int)min((int64_t)TILE, n - base);
        for (int i = threadIdx.x; i < NW * kOsMaxBins; i += NT) (&cnt[0][0])[i] = 0;
        K k[NI];
        uint32_t v[NI], r[NI];  // the digit is recomputed from the key (registers)
#pragma unroll
        for (int j = 0; j < NI; ++j) {  // wave w: records [w * 64 NI, (w + 1) * 64 NI), striped
            const int e = wave * (64 * NI) + j * 64 + lane;
            k[j] = e < cnt_t ? kin[base + e] : (K)0;
            if constexpr (V) v[j] = e < cnt_t ? (vin ? vin[base + e] : (uint32_t)(base + e)) : 0u;  // null: arrival index
        }
        __syncthreads();  // the counters are zero
#pragma unroll
        for (int j = 0; j < NI; ++j) {  // in order: stable within the wave
            const int e = wave * (64 * NI) + j * 64 + lane;
            const bool valid = e < cnt_t;
            const uint32_t dj = digit_of(k[j], shift, width);
            uint64_t peers = __ballot(valid);
            if (exp & 2) {
                r[j] = j * 64 + lane;
                continue;
            }
            for (int b = 0; b < width; ++b) {
                const bool bit = (dj >> b) & 1u;
                const uint64_t bb = __ballot(bit);
                peers &= bit ? bb : ~bb;
            }
            const uint32_t below = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
            uint32_t old = 0;
            if (valid && below == 0) {  // the group's lowest lane: only this wave writes its counters
                old = cnt[wave][dj];
                cnt[wave][dj] = old + (uint32_t)__popcll(peers);
            }
            old = __shfl(old, valid ? __ffsll((long long)peers) - 1 : lane);
            r[j] = old + below;
        }
        __syncthreads();
        // per digit: the waves' bases within the digit, the tile's count, its global position
        for (int b = threadIdx.x; b < nbins; b += NT) {
            uint32_t tot = 0;
#pragma unroll
            for (int w = 0; w < NW; ++w) {
                const uint32_t c = cnt[w][b];
                cnt[w][b] = tot;
                tot += c;
            }
            uint32_t* st = status + t * kOsMaxBins + b;
            if (t == 0) {
                __hip_atomic_store(st, tot | kOsIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gstart[b] = gbase[b];
            } else {
                __hip_atomic_store(st, tot | kOsLocal, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t excl = (exp & 1) ? 0u : os_look_back(status, t, b);
                __hip_atomic_store(st, (excl + tot) | kOsIncl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gstart[b] = gbase[b] + excl;
            }
            lstart[b] = tot;  // scanned below
        }
        __syncthreads();
        {  // exclusive scan of the tile's digit counts (<= 512: 512 / NT per thread)
            constexpr int PER = (kOsMaxBins + NT - 1) / NT;
            uint32_t a[PER], sum = 0;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int b = threadIdx.x * PER + i;
                a[i] = b < nbins ? lstart[b] : 0u;
                sum += a[i];
            }
            uint32_t incl = sum;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t up = __shfl_up(incl, o);
                if (lane >= o) incl += up;
            }
            if (lane == 63) wsum[wave] = incl;
            __syncthreads();
            uint32_t off = 0;
            for (int w = 0; w < wave; ++w) off += wsum[w];
            uint32_t ex = off + incl - sum;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int b = threadIdx.x * PER + i;
                if (b < nbins) lstart[b] = ex;
                ex += a[i];
            }
            if (threadIdx.x == NT - 1) lstart[nbins] = off + incl;
            __syncthreads();
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {  // reorder the tile by digit in LDS
            const int e = wave * (64 * NI) + j * 64 + lane;
            if (e < cnt_t) {
                const uint32_t dj = digit_of(k[j], shift, width);
                const uint32_t lp = lstart[dj] + cnt[wave][dj] + r[j];
                s_k[lp] = k[j];
                if constexpr (V) s_v[lp] = v[j];
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < cnt_t; i += NT) {  // out, bin run by bin run
            const K kk = s_k[i];
            const uint32_t dd = digit_of(kk, shift, width);
            const uint32_t at = gstart[dd] + (uint32_t)i - lstart[dd];
            if (exp & 4) {
                if (kk == 0xffffffffu) kout[0] = kk;
                continue;
            }
            kout[at] = kk;
            if constexpr (V) vout[at] = s_v[i];
        }
    }
}

__global__ void __launch_bounds__(256) k_iota(uint32_t* v, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[i] = (uint32_t)i;
}

// Tile shapes (GW_SORT_CFG picks one for the microbenchmark, scripts/r5/sortbench.cpp).  The
// defaults are the measured best on 10M records (profiles/r5/sort/): 512 x 12 for 4-B keys
// (3 x 9-bit passes over 26 bits: 0.249 ms; 256 x 16: 0.312, 512 x 8: 0.288), 512 x 8 for 8-B
// keys (40 bits: 0.507 ms; 512 x 12: 0.627).
struct OsCfg {
    int nt, ni, maxw;
};
static const OsCfg kOsCfgs[] = {{512, 12, 9}, {256, 16, 9}, {512, 16, 9}, {1024, 6, 9}, {512, 8, 9}, {384, 16, 9}};
static OsCfg os_cfg(int key_bytes) {
    static const int c = getenv("GW_SORT_CFG") ? atoi(getenv("GW_SORT_CFG")) : -1;
    if (c >= 0 && c < (int)(sizeof kOsCfgs / sizeof kOsCfgs[0])) return kOsCfgs[c];
    return key_bytes == 8 ? kOsCfgs[4] : kOsCfgs[0];
}
static int64_t os_tiles(int64_t n, int tile) { return n <= 0 ? 0 : (n + tile - 1) / tile; }

// scratch: ghist[8][512] (+ 64 words), two look-back regions
constexpr int kOsHead = 8 * kOsMaxBins + 64;
int64_t sort_scratch_bytes(int64_t n) {
    return (kOsHead + 2 * os_tiles(std::max<int64_t>(n, 1), 256 * 12) * kOsMaxBins) * 4 + 256;
}
int64_t radix_sort_scratch_bytes(int64_t n) { return sort_scratch_bytes(n); }

static int num_cus() {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        cus = std::max(1, cus);
    }
    return cus;
}

template <typename K, bool V, int NT, int NI>
static hipError_t os_launch(const K* kin, const uint32_t* vin, K* kout, uint32_t* vout, int64_t n, int shift, int width,
                            const uint32_t* gbase, uint32_t* status, uint32_t* next_status, int64_t nt,
                            uint32_t* tile_ctr, hipStream_t s) {
    hipLaunchKernelGGL((k_os_pass<K, V, NT, NI>), dim3((unsigned)nt), dim3(NT), 0, s, kin, vin, kout, vout, n, shift,
                       width, gbase, status, next_status, nt, tile_ctr);
    return hipGetLastError();
}

template <typename K, bool V>
static hipError_t os_pass(const OsCfg& c, const K* kin, const uint32_t* vin, K* kout, uint32_t* vout, int64_t n,
                          int shift, int width, const uint32_t* gbase, uint32_t* status, uint32_t* next_status,
                          int64_t nt, uint32_t* tile_ctr, hipStream_t s) {
#define OS(NT, NI) \
    return os_launch<K, V, NT, NI>(kin, vin, kout, vout, n, shift, width, gbase, status, next_status, nt, tile_ctr, s)
    if (c.nt == 256 && c.ni == 16) OS(256, 16);
    if (c.nt == 512 && c.ni == 16) OS(512, 16);
    if (c.nt == 1024 && c.ni == 6) OS(1024, 6);
    if (c.nt == 512 && c.ni == 8) OS(512, 8);
    if (c.nt == 384 && c.ni == 16) OS(384, 16);
    OS(512, 12);
#undef OS
}

// iota: v0's contents are not read; the values are the arrival indices 0..n-1 (the first pass
// makes them).
template <typename K>
static hipError_t sort_pairs_impl(K* k0, uint32_t* v0, K* k1, uint32_t* v1, int64_t n, int lo, int hi, void* scratch,
                                  hipStream_t s, int* result_in_alt, bool iota) {
    *result_in_alt = 0;
    if (n > kSortMaxRecords) return hipErrorInvalidValue;  // the 30-bit prefix field would spill into the flags
    const OsCfg c = os_cfg((int)sizeof(K));
    const SortPlan p = plan_for(lo, hi, c.maxw);
    if (n <= 1 || p.npass == 0) return iota && n > 0 ? launch_iota(v0, n, s) : hipSuccess;
    uint32_t* ghist = (uint32_t*)scratch;
    const int64_t nt = os_tiles(n, c.nt * c.ni);
    uint32_t* region[2] = {ghist + kOsHead, ghist + kOsHead + nt * kOsMaxBins};
    // ghist and the first pass's look-back words; each pass zeroes the next pass's
    hipError_t e = hipMemsetAsync(ghist, 0, (size_t)(kOsHead + nt * kOsMaxBins) * 4, s);
    if (e != hipSuccess) return e;
    const int hg = (int)std::min<int64_t>(2 * num_cus(), (n + 4095) / 4096);
    hipLaunchKernelGGL(k_os_hist<K>, dim3(std::max(1, hg)), dim3(1024), 0, s, (const K*)k0, n, p, ghist);
    hipLaunchKernelGGL(k_os_scan, dim3(1), dim3(512), 0, s, ghist, p.npass);
    int alt = 0;
    for (int q = 0; q < p.npass; ++q) {
        K* kin = alt ? k1 : k0;
        K* kout = alt ? k0 : k1;
        uint32_t* vin = alt ? v1 : (iota && q == 0 ? nullptr : v0);
        uint32_t* vout = alt ? v0 : v1;
        uint32_t* st = region[q & 1];
        uint32_t* nx = q + 1 < p.npass ? region[(q + 1) & 1] : nullptr;
        uint32_t* ctr = ghist + 8 * kOsMaxBins + q;  // zeroed with ghist
        e = v0 ? os_pass<K, true>(c, kin, vin, kout, vout, n, p.shift[q], p.width[q], ghist + q * kOsMaxBins,
                                          st, nx, nt, ctr, s)
                       : os_pass<K, false>(c, kin, nullptr, kout, nullptr, n, p.shift[q], p.width[q],
                                           ghist + q * kOsMaxBins, st, nx, nt, ctr, s);
        if (e != hipSuccess) return e;
        alt ^= 1;
    }
    *result_in_alt = alt;
    return hipGetLastError();
}

hipError_t sort_pairs_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, int64_t n, int lo, int hi,
                          void* scratch, hipStream_t s, int* result_in_alt, bool iota) {
    return sort_pairs_impl<uint32_t>(k0, v0, k1, v1, n, lo, hi, scratch, s, result_in_alt, iota && v0);
}
hipError_t sort_pairs_u64(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, int64_t n, int lo, int hi,
                          void* scratch, hipStream_t s, int* result_in_alt, bool iota) {
    return sort_pairs_impl<uint64_t>(k0, v0, k1, v1, n, lo, hi, scratch, s, result_in_alt, iota && v0);
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
