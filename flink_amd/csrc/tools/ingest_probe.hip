// ingest_probe.hip — microbenchmark of the ingest kernel's cost components on gfx950.
// Not part of the library.  Build: hipcc --offload-arch=gfx950 -O3 -munsafe-fp-atomics
//   flink_amd/csrc/tools/ingest_probe.hip -o flink_amd/_build/ingest_probe
// Table: 2^24 slots x 64 B (1 GiB) holding 10M keys; batch: 10M events, uniform keys.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../gw_device.h"

using namespace gw;

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

__device__ unsigned long long g_sink;

__global__ void k_fill_keys(int64_t* keys, int64_t n, int64_t K, uint64_t seed) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        keys[i] = (int64_t)((z >> 1) % (uint64_t)K);
    }
}

__global__ void k_init(TableView t) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= t.cap; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t* s = slot_ptr(t, i);
        s[0] = kEmptyKey;
        for (int w = 1; w < t.stride_w; ++w) s[w] = 0;
    }
}

__global__ void k_insert(TableView t, const int64_t* keys, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool ins;
        find_or_insert(t, keys[i], ins);
    }
}

template <int V>
__global__ void __launch_bounds__(256) k_variant(TableView t, const int64_t* key, const int64_t* ts,
                                                 const int64_t* val, int64_t n) {
    unsigned long long acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = key[i];
        const int64_t tt = ts[i];
        const int64_t v = val[i];
        const uint32_t pos = (uint32_t)(tt & 3);
        if constexpr (V == 0) {  // stream only
            acc += (unsigned long long)(k ^ tt ^ v) + slot_hash(k);
        } else if constexpr (V == 10) {  // random 8-B gather from the table (no probing)
            const uint64_t idx = slot_hash(k) & (uint64_t)(t.cap - 1);
            acc += (unsigned long long)slot_ptr(t, idx)[0];
        } else if constexpr (V == 11) {  // random device atomic add, no read
            const uint64_t idx = slot_hash(k) & (uint64_t)(t.cap - 1);
            atomicAdd((unsigned long long*)(slot_ptr(t, idx) + 2 + pos), (unsigned long long)v);
        } else {
            bool ins;
            const int64_t si = find_or_insert(t, k, ins);
            int64_t* s = slot_ptr(t, si);
            if constexpr (V == 1) {  // probe only
                acc += (unsigned long long)si;
            } else if constexpr (V == 2) {  // probe + plain RMW (racy; timing only)
                s[2 + pos] += v;
            } else if constexpr (V == 3) {  // probe + atomic add
                atomicAdd((unsigned long long*)(s + 2 + pos), (unsigned long long)v);
            } else if constexpr (V == 4) {  // probe + atomic add + conditional mask OR (= k_ingest)
                atomicAdd((unsigned long long*)(s + 2 + pos), (unsigned long long)v);
                const unsigned long long bit = 1ull << pos;
                if (!(*(volatile unsigned long long*)(s + 1) & bit)) atomicOr((unsigned long long*)(s + 1), bit);
            } else if constexpr (V == 5) {  // probe + agent-scope relaxed atomic via builtin
                __hip_atomic_fetch_add((unsigned long long*)(s + 2 + pos), (unsigned long long)v,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if constexpr (V == 6) {  // probe + workgroup-scope atomic (performed in L2; racy across XCDs)
                __hip_atomic_fetch_add((unsigned long long*)(s + 2 + pos), (unsigned long long)v,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    if (acc == 0x1234567) g_sink = acc;
}

template <int V>
float run(TableView t, const int64_t* k, const int64_t* ts, const int64_t* v, int64_t n, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_variant<V>, dim3(grid), dim3(256), 0, 0, t, k, ts, v, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    const int64_t cap = 1 << 24, n = 10'000'000, K = 10'000'000;
    TableView t{};
    t.cap = cap;
    t.stride_w = 8;
    t.ring = 6;
    t.words = 1;
    CK(hipMalloc((void**)&t.base, (size_t)(cap + 1) * 64));
    int64_t *k, *ts, *v;
    CK(hipMalloc((void**)&k, n * 8));
    CK(hipMalloc((void**)&ts, n * 8));
    CK(hipMalloc((void**)&v, n * 8));
    hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, t);
    hipLaunchKernelGGL(k_fill_keys, dim3(4096), dim3(256), 0, 0, k, n, K, 1);
    hipLaunchKernelGGL(k_fill_keys, dim3(4096), dim3(256), 0, 0, ts, n, 1000, 2);
    hipLaunchKernelGGL(k_fill_keys, dim3(4096), dim3(256), 0, 0, v, n, 1000000, 3);
    // pre-insert all keys 0..K-1
    int64_t* all;
    CK(hipMalloc((void**)&all, K * 8));
    std::vector<int64_t> h(K);
    for (int64_t i = 0; i < K; ++i) h[i] = i;
    CK(hipMemcpy(all, h.data(), K * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_insert, dim3(4096), dim3(256), 0, 0, t, all, K);
    CK(hipDeviceSynchronize());
    const char* names[] = {"stream only (24 B/event)", "probe only", "probe + plain RMW (racy)",
                           "probe + atomicAdd", "probe + atomicAdd + mask OR (k_ingest)",
                           "probe + agent relaxed fetch_add", "probe + workgroup-scope atomic (L2)"};
    for (int grid : {1024, 4096, 16384}) {
        printf("grid %d blocks x 256\n", grid);
        float ms[12];
        ms[0] = run<0>(t, k, ts, v, n, grid);
        ms[1] = run<1>(t, k, ts, v, n, grid);
        ms[2] = run<2>(t, k, ts, v, n, grid);
        ms[3] = run<3>(t, k, ts, v, n, grid);
        ms[4] = run<4>(t, k, ts, v, n, grid);
        ms[5] = run<5>(t, k, ts, v, n, grid);
        ms[6] = run<6>(t, k, ts, v, n, grid);
        for (int i = 0; i < 7; ++i)
            printf("  V%d %-42s %8.3f ms  %7.2f Gev/s  stream-equiv %7.1f GB/s\n", i, names[i], ms[i],
                   n / ms[i] / 1e6, n * 24.0 / ms[i] / 1e6);
        float g10 = run<10>(t, k, ts, v, n, grid), g11 = run<11>(t, k, ts, v, n, grid);
        printf("  V10 random 8-B gather only              %8.3f ms  %7.2f Gev/s\n", g10, n / g10 / 1e6);
        printf("  V11 random atomicAdd only (no read)     %8.3f ms  %7.2f Gev/s\n", g11, n / g11 / 1e6);
    }
    return 0;
}
