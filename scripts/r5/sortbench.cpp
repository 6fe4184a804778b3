// Microbenchmark of gw_sort.hip's sort_pairs_u32 / sort_pairs_u64: n random keys of `bits` bits
// with arrival indices, timed per sort with HIP events, checked once against std::stable_sort.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I flink_amd/csrc scripts/r5/sortbench.cpp \
//         flink_amd/csrc/gw_sort.hip -o scripts/r5/sortbench
//   scripts/r5/sortbench [n] [bits] [reps] [u64] [iota]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#include "gw_sort.h"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

template <typename K>
static int run(int64_t n, int bits, int reps, bool iota) {
    std::mt19937_64 rng(7);
    std::vector<K> hk(n);
    for (auto& k : hk) k = (K)(rng() & ((bits >= 64 ? ~0ull : (1ull << bits) - 1)));
    std::vector<uint32_t> hv(n);
    std::iota(hv.begin(), hv.end(), 0u);
    K *k0, *k1;
    uint32_t *v0, *v1;
    void* scratch;
    CK(hipMalloc(&k0, n * sizeof(K)));
    CK(hipMalloc(&k1, n * sizeof(K)));
    CK(hipMalloc(&v0, n * 4));
    CK(hipMalloc(&v1, n * 4));
    CK(hipMalloc(&scratch, gw::sort_scratch_bytes(n)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ms;
    int alt = 0;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipMemcpy(k0, hk.data(), n * sizeof(K), hipMemcpyHostToDevice));
        if (iota)
            CK(hipMemset(v0, 0xab, n * 4));
        else
            CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipEventRecord(a, 0));
        if constexpr (sizeof(K) == 4)
            CK(gw::sort_pairs_u32(k0, v0, k1, v1, n, 0, bits, scratch, 0, &alt, iota));
        else
            CK(gw::sort_pairs_u64(k0, v0, k1, v1, n, 0, bits, scratch, 0, &alt, iota));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t = 0;
        CK(hipEventElapsedTime(&t, a, b));
        if (r >= 2) ms.push_back(t);
    }
    std::vector<K> gk(n);
    std::vector<uint32_t> gv(n);
    CK(hipMemcpy(gk.data(), alt ? k1 : k0, n * sizeof(K), hipMemcpyDeviceToHost));
    CK(hipMemcpy(gv.data(), alt ? v1 : v0, n * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return hk[x] < hk[y]; });
    int64_t bad = 0;
    for (int64_t i = 0; i < n; ++i)
        if (gv[i] != idx[i] || gk[i] != hk[idx[i]]) ++bad;
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    const double bytes = (double)n * (sizeof(K) + 4) * 2 * ((bits + 8) / 9);
    printf("{\"n\": %lld, \"bits\": %d, \"key_bytes\": %d, \"median_ms\": %.4f, \"min_ms\": %.4f, "
           "\"pass_GBps\": %.1f, \"mismatches\": %lld}\n",
           (long long)n, bits, (int)sizeof(K), med, ms[0], bytes / med / 1e6, (long long)bad);
    return bad ? 2 : 0;
}

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
    const int bits = argc > 2 ? atoi(argv[2]) : 25;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const bool u64 = argc > 4 && atoi(argv[4]);
    const bool iota = argc > 5 && atoi(argv[5]);
    return u64 ? run<uint64_t>(n, bits, reps, iota) : run<uint32_t>(n, bits, reps, iota);
}
