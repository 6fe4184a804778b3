// gw_sort.hip — hand-written LSD radix sort (uint64 keys, uint32 payload) for gfx950.
//
// Used by the session path to group a batch by (state slot, timestamp): the GPU
// analogue of MergingWindowSet's per-key sorted window list (reference:
// TimeWindow.mergeWindows sorts by start, RS/api/windowing/windows/TimeWindow.java:208-254).
// 8-bit digits; per pass: block histogram (LDS atomics) -> one-block scan ->
// stable scatter with wave64 ballot matching (8 ballots give each lane the mask of
// same-digit lanes in its wave; in-wave rank = popcount below the lane).
#include "gw_sort.h"

namespace gw {

constexpr int kRsThreads = 256;
constexpr int kRsItems = 16;
constexpr int kRsTile = kRsThreads * kRsItems;

static int64_t rs_blocks(int64_t n) { return n <= 0 ? 1 : (n + kRsTile - 1) / kRsTile; }

__global__ void __launch_bounds__(256) k_rs_hist(const uint64_t* keys, int64_t n, int shift, uint32_t* counts) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kRsTile;
#pragma unroll 4
    for (int r = 0; r < kRsItems; ++r) {
        const int64_t i = t0 + (int64_t)r * kRsThreads + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    counts[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of counts[256][nb] (bin-major) into offsets (same layout)
__global__ void __launch_bounds__(1024) k_rs_scan(const uint32_t* counts, int64_t total, uint32_t* offsets) {
    __shared__ uint32_t part[1024];
    const int64_t per = (total + blockDim.x - 1) / blockDim.x;
    const int64_t lo = threadIdx.x * per, hi = min(total, lo + per);
    uint32_t s = 0;
    for (int64_t i = lo; i < hi; ++i) s += counts[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
        uint32_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (int64_t i = lo; i < hi; ++i) { uint32_t v = counts[i]; offsets[i] = run; run += v; }
}

__global__ void __launch_bounds__(256) k_rs_scatter(const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                                    uint32_t* vout, int64_t n, int shift, const uint32_t* offsets) {
    __shared__ uint32_t run[256];
    __shared__ uint32_t wc[4][256];
    const int lane = __lane_id();
    const int wave = threadIdx.x >> 6;
    run[threadIdx.x] = offsets[(int64_t)threadIdx.x * gridDim.x + blockIdx.x];
    const int64_t t0 = (int64_t)blockIdx.x * kRsTile;
    for (int r = 0; r < kRsItems; ++r) {
        wc[0][threadIdx.x] = 0; wc[1][threadIdx.x] = 0; wc[2][threadIdx.x] = 0; wc[3][threadIdx.x] = 0;
        __syncthreads();
        const int64_t i = t0 + (int64_t)r * kRsThreads + threadIdx.x;
        const bool valid = i < n;
        uint64_t k = 0;
        uint32_t v = 0;
        uint32_t d = 0;
        if (valid) { k = kin[i]; v = vin ? vin[i] : 0u; d = (uint32_t)(k >> shift) & 255u; }
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (valid && rank == 0) wc[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = run[d] + rank;
            for (int w = 0; w < wave; ++w) pos += wc[w][d];
            kout[pos] = k;
            if (vout) vout[pos] = v;
        }
        __syncthreads();
        run[threadIdx.x] += wc[0][threadIdx.x] + wc[1][threadIdx.x] + wc[2][threadIdx.x] + wc[3][threadIdx.x];
    }
}

__global__ void __launch_bounds__(256) k_iota(uint32_t* v, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[i] = (uint32_t)i;
}

int64_t radix_sort_scratch_bytes(int64_t n) {
    const int64_t nb = rs_blocks(n);
    return 2 * 256 * nb * (int64_t)sizeof(uint32_t) + 256;
}

hipError_t radix_sort_pairs(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, int64_t n, int bits,
                            void* scratch, hipStream_t s, int* result_in_alt) {
    const int64_t nb = rs_blocks(n);
    uint32_t* counts = (uint32_t*)scratch;
    uint32_t* offs = counts + 256 * nb;
    int alt = 0;
    for (int shift = 0; shift < bits; shift += 8) {
        const uint64_t* kin = alt ? k1 : k0;
        const uint32_t* vin = alt ? v1 : v0;
        uint64_t* kout = alt ? k0 : k1;
        uint32_t* vout = alt ? v0 : v1;
        hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)nb), dim3(256), 0, s, kin, n, shift, counts);
        hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(1024), 0, s, counts, 256 * nb, offs);
        hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)nb), dim3(256), 0, s, kin, vin, kout, vout, n, shift, offs);
        alt ^= 1;
    }
    *result_in_alt = alt;
    return hipGetLastError();
}

hipError_t launch_iota(uint32_t* v, int64_t n, hipStream_t s) {
    int64_t g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(k_iota, dim3((unsigned)g), dim3(256), 0, s, v, n);
    return hipGetLastError();
}

}  // namespace gw
