// gw_select.hip — a stable filter + dictionary lookup ahead of the window operator.
//
// The stages a job runs before keyBy on simple records: FilterFunction (keep the records
// whose selector column equals one value), a projection, and a join against a static
// dictionary (the Yahoo Streaming Benchmark's ad -> campaign lookup, Redis in the original
// AdvertisingTopologyNative).  Flink runs them as chained operators in front of the window
// operator; on the device they are one read of the columns and one write of the survivors.
//
// Three launches over tiles of kSelTile records: per-tile match counts (reads the selector
// only), a one-block exclusive scan of the counts, and the stable scatter (wave ballots rank
// each match within its tile; item j of thread x is record tile_base + j * 256 + x, so the
// loads coalesce and the ranks follow arrival order).
#include "gw_kernels.h"

#include <algorithm>

namespace gw {

constexpr int kSelThreads = 256, kSelItems = 16, kSelTile = kSelThreads * kSelItems;

__global__ void __launch_bounds__(kSelThreads) k_sel_count(int64_t n, const int64_t* sel, int64_t want,
                                                           uint32_t* tile_cnt) {
    __shared__ uint32_t s_cnt[kSelThreads / 64];
    const int64_t base = (int64_t)blockIdx.x * kSelTile;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kSelItems; ++j) {
        const int64_t i = base + j * kSelThreads + threadIdx.x;
        c += (i < n && sel[i] == want) ? 1u : 0u;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (__lane_id() == 0) s_cnt[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kSelThreads / 64; ++w) t += s_cnt[w];
        tile_cnt[blockIdx.x] = t;
    }
}

// One block: exclusive scan of ntiles counts into tile_off, the total into *total.
__global__ void __launch_bounds__(1024) k_sel_scan(const uint32_t* tile_cnt, int64_t ntiles, int64_t* tile_off,
                                                   int64_t* total) {
    __shared__ int64_t s_w[1024 / 64];
    __shared__ int64_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = __lane_id(), w = threadIdx.x >> 6;
    for (int64_t t0 = 0; t0 < ntiles; t0 += blockDim.x) {
        const int64_t t = t0 + threadIdx.x;
        const int64_t v = t < ntiles ? (int64_t)tile_cnt[t] : 0;
        int64_t incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t up = __shfl_up(incl, o);
            if (lane >= o) incl += up;
        }
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        int64_t off = s_carry;
        for (int q = 0; q < w; ++q) off += s_w[q];
        if (t < ntiles) tile_off[t] = off + incl - v;
        __syncthreads();
        if (threadIdx.x == blockDim.x - 1) s_carry = off + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = s_carry;
}

__global__ void __launch_bounds__(kSelThreads) k_sel_scatter(int64_t n, const int64_t* sel, int64_t want,
                                                             const int64_t* idx, const int64_t* dict, int64_t dict_n,
                                                             const int64_t* ts, const int64_t* tile_off,
                                                             int64_t* key_out, int64_t* ts_out, int32_t* bad) {
    constexpr int kW = kSelThreads / 64;
    __shared__ uint32_t s_cnt[kSelItems][kW];
    const int lane = __lane_id(), w = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kSelTile;
    bool hit[kSelItems];
    uint32_t before[kSelItems];
#pragma unroll
    for (int j = 0; j < kSelItems; ++j) {
        const int64_t i = base + j * kSelThreads + threadIdx.x;
        hit[j] = i < n && sel[i] == want;
        const unsigned long long b = __ballot(hit[j]);
        before[j] = (uint32_t)__popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) s_cnt[j][w] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // exclusive scan over (item, wave): arrival order within the tile
        uint32_t run = 0;
        for (int j = 0; j < kSelItems; ++j)
            for (int q = 0; q < kW; ++q) {
                const uint32_t c = s_cnt[j][q];
                s_cnt[j][q] = run;
                run += c;
            }
    }
    __syncthreads();
    const int64_t off = tile_off[blockIdx.x];
    int32_t oob = 0;
#pragma unroll
    for (int j = 0; j < kSelItems; ++j) {
        if (!hit[j]) continue;
        const int64_t i = base + j * kSelThreads + threadIdx.x;
        const int64_t o = off + s_cnt[j][w] + before[j];
        const int64_t x = idx[i];
        const bool ok = x >= 0 && x < dict_n;
        oob |= ok ? 0 : 1;
        key_out[o] = ok ? dict[x] : 0;
        ts_out[o] = ts[i];
    }
    if (__any(oob) && lane == 0) atomicOr(bad, 1);
}

hipError_t launch_select_lookup(int64_t n, const int64_t* sel, int64_t want, const int64_t* idx, const int64_t* dict,
                                int64_t dict_n, const int64_t* ts, int64_t* key_out, int64_t* ts_out, void* scratch,
                                hipStream_t s) {
    const int64_t ntiles = (n + kSelTile - 1) / kSelTile;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(scratch);
    int64_t* off = reinterpret_cast<int64_t*>(reinterpret_cast<char*>(scratch) + ((ntiles * 4 + 15) / 16) * 16);
    int64_t* total = off + ntiles;
    int32_t* bad = reinterpret_cast<int32_t*>(total + 1);
    hipError_t e = hipMemsetAsync(bad, 0, 4, s);
    if (e != hipSuccess) return e;
    if (ntiles > 0) {
        hipLaunchKernelGGL(k_sel_count, dim3((unsigned)ntiles), dim3(kSelThreads), 0, s, n, sel, want, cnt);
    }
    hipLaunchKernelGGL(k_sel_scan, dim3(1), dim3(1024), 0, s, cnt, ntiles, off, total);
    if (ntiles > 0) {
        hipLaunchKernelGGL(k_sel_scatter, dim3((unsigned)ntiles), dim3(kSelThreads), 0, s, n, sel, want, idx, dict,
                           dict_n, ts, off, key_out, ts_out, bad);
    }
    return hipGetLastError();
}

size_t select_lookup_scratch_bytes(int64_t n) {
    const int64_t ntiles = (n + kSelTile - 1) / kSelTile;
    return (size_t)((ntiles * 4 + 15) / 16) * 16 + (size_t)(ntiles + 2) * 8;
}

}  // namespace gw
