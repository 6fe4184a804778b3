// mall_probe.hip — random gather / atomic rates vs. footprint on gfx950 (Infinity Cache
// residency study for the state-table layout).  Not part of the library.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

__device__ unsigned long long g_sink;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

__global__ void k_fill(int64_t* keys, int64_t n, int64_t K) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        keys[i] = (int64_t)(mix((uint64_t)i * 0x9E3779B97F4A7C15ull + 7) % (uint64_t)K);
}

// MODE 0: gather A[h]; 1: atomicAdd B[h]; 2: gather A[h] then atomicAdd B[h]; 3: = 2 with nt stream loads;
// 4: gather A[h] + plain RMW B[h] (racy); 5: gather + atomic + atomicOr bitmap
template <int MODE>
__global__ void __launch_bounds__(256) k_rand(const int64_t* key, const int64_t* val, int64_t n, int64_t* A, int64_t* B,
                                              unsigned long long* bits, uint64_t slots, int stride_w) {
    unsigned long long acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t k, v;
        if constexpr (MODE == 3) {
            k = __builtin_nontemporal_load(key + i);
            v = __builtin_nontemporal_load(val + i);
        } else {
            k = key[i];
            v = val[i];
        }
        const uint64_t h = mix((uint64_t)k) % slots;
        if constexpr (MODE == 0) acc += (unsigned long long)A[h * stride_w];
        if constexpr (MODE == 1) atomicAdd((unsigned long long*)&B[h * stride_w], (unsigned long long)v);
        if constexpr (MODE == 2 || MODE == 3 || MODE == 5) {
            if (A[h * stride_w] == k + 1) acc++;
            atomicAdd((unsigned long long*)&B[h * stride_w], (unsigned long long)v);
        }
        if constexpr (MODE == 5) {
            const unsigned long long bit = 1ull << (h & 63);
            unsigned long long* w = bits + (h >> 6);
            if (!(*(volatile unsigned long long*)w & bit)) atomicOr(w, bit);
        }
        if constexpr (MODE == 4) {
            if (A[h * stride_w] == k + 1) acc++;
            B[h * stride_w] += v;
        }
    }
    if (acc == 0x12345) g_sink = acc;
}

template <int MODE>
float run(const int64_t* k, const int64_t* v, int64_t n, int64_t* A, int64_t* B, unsigned long long* bits,
          uint64_t slots, int sw) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_rand<MODE>, dim3(8192), dim3(256), 0, 0, k, v, n, A, B, bits, slots, sw);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (r > 0 && ms < best) best = ms;
    }
    return best;
}

int main() {
    const int64_t n = 10'000'000;
    int64_t *k, *v;
    CK(hipMalloc((void**)&k, n * 8));
    CK(hipMalloc((void**)&v, n * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, k, n, 10'000'000);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, v, n, 1000);
    const size_t big = (size_t)2 << 30;
    int64_t *A, *B;
    unsigned long long* bits;
    CK(hipMalloc((void**)&A, big));
    CK(hipMalloc((void**)&B, big));
    CK(hipMalloc((void**)&bits, 64 << 20));
    CK(hipMemset(A, 0, big));
    CK(hipMemset(B, 0, big));
    CK(hipMemset(bits, 0, 64 << 20));
    CK(hipDeviceSynchronize());
    struct Cfg { uint64_t slots; int sw; };
    Cfg cfgs[] = {{4u << 20, 1}, {8u << 20, 1}, {12'500'000, 1}, {16u << 20, 1}, {32u << 20, 1}, {16u << 20, 8}};
    printf("%-26s %10s %10s %10s %10s %10s %10s   (G events/s, 10M events)\n", "footprint per array", "gather",
           "atomic", "gath+atom", "nt-stream", "plainRMW", "+bitmap");
    for (auto c : cfgs) {
        float m0 = run<0>(k, v, n, A, B, bits, c.slots, c.sw);
        float m1 = run<1>(k, v, n, A, B, bits, c.slots, c.sw);
        float m2 = run<2>(k, v, n, A, B, bits, c.slots, c.sw);
        float m3 = run<3>(k, v, n, A, B, bits, c.slots, c.sw);
        float m4 = run<4>(k, v, n, A, B, bits, c.slots, c.sw);
        float m5 = run<5>(k, v, n, A, B, bits, c.slots, c.sw);
        char lab[64];
        snprintf(lab, sizeof(lab), "%llu slots x %d B", (unsigned long long)c.slots, 8 * c.sw);
        printf("%-26s %10.2f %10.2f %10.2f %10.2f %10.2f %10.2f   [%.0f MB/array]\n", lab, n / m0 / 1e6, n / m1 / 1e6,
               n / m2 / 1e6, n / m3 / 1e6, n / m4 / 1e6, n / m5 / 1e6, c.slots * 8.0 * c.sw / 1e6);
    }
    return 0;
}
