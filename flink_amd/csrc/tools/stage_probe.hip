// stage_probe.hip -- does a staging buffer written by one kernel and read back by the next
// stay on-die (XCD L2 / Infinity Cache) on gfx950?  Decides whether the region path's second
// partition level can read pass 1's output without an HBM round trip.  Not part of the library.
//
//   hipcc -O3 --offload-arch=gfx950 stage_probe.hip -o stage_probe && ./stage_probe
//
// For staging sizes S: kernel W writes S bytes (16 B per lane, workgroup g owns chunk g),
// optionally kernel X streams Y bytes of unrelated input (non-temporal loads, as pass 1 reads
// its batch), then kernel R reads the S bytes back: with the same chunk -> workgroup map
// (same XCD as the writer) or shifted by one workgroup (another XCD).  R's time against a cold
// read of a buffer nobody touched recently says where the bytes came from.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); }     \
    } while (0)

__device__ unsigned long long g_sink;
constexpr int kBlocks = 2048, kThreads = 256;
typedef long long v2 __attribute__((ext_vector_type(2)));

template <int NT>
__global__ void __launch_bounds__(kThreads) k_write(v2* p, int64_t n16, int64_t salt) {
    const int64_t per = (n16 + kBlocks - 1) / kBlocks;
    const int64_t lo = blockIdx.x * per, hi = lo + per < n16 ? lo + per : n16;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
        const v2 v{i ^ salt, i + salt};
        if (NT) __builtin_nontemporal_store(v, p + i);
        else p[i] = v;
    }
}

template <int NT>
__global__ void __launch_bounds__(kThreads) k_read(const v2* p, int64_t n16, int shift) {
    const int64_t per = (n16 + kBlocks - 1) / kBlocks;
    const int64_t b = (blockIdx.x + shift) % kBlocks;
    const int64_t lo = b * per, hi = lo + per < n16 ? lo + per : n16;
    long long acc = 0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
        const v2 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
        acc += v.x ^ v.y;
    }
    if (acc == 0x123456789) g_sink = acc;
}

int main() {
    const size_t maxS = (size_t)1 << 30, maxY = (size_t)1 << 30, cold = (size_t)2 << 30;
    v2 *S, *Y, *C;
    CK(hipMalloc((void**)&S, maxS));
    CK(hipMalloc((void**)&Y, maxY));
    CK(hipMalloc((void**)&C, cold));
    CK(hipMemset(S, 1, maxS));
    CK(hipMemset(Y, 2, maxY));
    CK(hipMemset(C, 3, cold));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timed = [&](auto launch) {
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        return ms;
    };
    // flush the caches: stream the 2-GB cold buffer
    auto flush = [&]() { hipLaunchKernelGGL(k_read<1>, dim3(kBlocks), dim3(kThreads), 0, 0, C, (int64_t)(cold / 16), 0); };
    printf("%8s %8s %3s %5s | %9s %9s | %9s (GB/s of the read-back; W = write rate)\n", "S_MB", "Y_MB", "nt", "shift",
           "read", "W", "cold");
    const size_t sizes[] = {8u << 20, 24u << 20, 64u << 20, 128u << 20, 200u << 20, 512u << 20};
    const size_t ys[] = {0, 48u << 20, 240u << 20, 512u << 20};
    for (size_t s : sizes) {
        const int64_t n16 = (int64_t)(s / 16);
        // cold read of S
        float cbest = 1e9f;
        for (int r = 0; r < 3; ++r) {
            flush();
            cbest = fminf(cbest, timed([&] { hipLaunchKernelGGL(k_read<0>, dim3(kBlocks), dim3(kThreads), 0, 0, S, n16, 0); }));
        }
        for (int nt = 0; nt < 2; ++nt)
            for (size_t y : ys)
                for (int shift = 0; shift < 2; ++shift) {
                    float rbest = 1e9f, wbest = 1e9f;
                    for (int r = 0; r < 3; ++r) {
                        flush();
                        const float w = timed([&] {
                            if (nt) hipLaunchKernelGGL(k_write<1>, dim3(kBlocks), dim3(kThreads), 0, 0, S, n16, (int64_t)r);
                            else hipLaunchKernelGGL(k_write<0>, dim3(kBlocks), dim3(kThreads), 0, 0, S, n16, (int64_t)r);
                        });
                        if (y) hipLaunchKernelGGL(k_read<1>, dim3(kBlocks), dim3(kThreads), 0, 0, Y, (int64_t)(y / 16), 0);
                        const float rd =
                            timed([&] { hipLaunchKernelGGL(k_read<0>, dim3(kBlocks), dim3(kThreads), 0, 0, S, n16, shift); });
                        rbest = fminf(rbest, rd);
                        wbest = fminf(wbest, w);
                    }
                    printf("%8zu %8zu %3d %5d | %9.0f %9.0f | %9.0f\n", s >> 20, y >> 20, nt, shift, s / rbest / 1e6,
                           s / wbest / 1e6, s / cbest / 1e6);
                }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
