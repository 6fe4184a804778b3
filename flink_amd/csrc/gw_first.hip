// gw_first.hip — first-element rows for positional aggregations (GW_FLAG_FIRST_ELEMENT).
//
// WindowedStream.sum(i) / min(i) / max(i) reduce with SumAggregator / ComparableAggregator
// (RS/api/functions/aggregation/SumAggregator.java:66-76, ComparableAggregator.java:83-104):
// the window's state is a copy of its FIRST element (in arrival order) with the aggregated
// field replaced, so the emitted tuple carries the first element's other fields.  The handle
// runs two operators over the same records (gw_runtime.cpp): A folds the aggregate, B folds
// MIN over each record's arrival sequence number; both fire the same (key, window) set.  At
// drain time their rows are joined by (key, window start) -- a stable LSD radix sort of each
// side by start, then by key -- and B's minimum sequence indexes the payload log (the other
// fields of every record, packed by the caller into one 64-bit word, kept until all windows
// that could hold the record are cleaned).
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

#include "gw_first.h"

namespace gw {

__global__ void k_fe_iota64(int64_t* d, int64_t n, int64_t base) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = base + i;
}

__global__ void k_fe_iota32(uint32_t* d, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = (uint32_t)i;
}

__global__ void k_fe_gather_key(const int64_t* src, const uint32_t* idx, int64_t* dst, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[idx[i]];
}

// The batch's largest timestamp: wave then block reduction, one device atomic per block
// (a small grid: thousands of atomics on one address serialise at the memory side).
__global__ void __launch_bounds__(256) k_fe_max(const int64_t* ts, int64_t n, int64_t* out) {
    __shared__ int64_t wmax[4];
    int64_t m = INT64_MIN;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        m = max(m, ts[i]);
    for (int o = 32; o > 0; o >>= 1) m = max(m, (int64_t)__shfl_xor(m, o));
    if (__lane_id() == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (m != INT64_MIN) atomicMax((long long*)out, (long long)m);
    }
}

// n payloads to log positions [at, at + n) (the host splits a ring wrap into two calls)
__global__ void k_fe_append(int64_t* log, int64_t at, const int64_t* src, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        log[at + i] = src[i];
}

// Row i of the join: A's row pa[i] and B's row pb[i] (both sorted by (key, start)).
__global__ void k_fe_zip(int64_t n, const uint32_t* pa, const uint32_t* pb, const int64_t* a_key,
                         const int64_t* a_start, const int64_t* a_end, const int64_t* a_res, const int64_t* b_key,
                         const int64_t* b_start, const int64_t* b_res, const int64_t* log, int64_t log_base,
                         int64_t log_cap, int64_t* o_key, int64_t* o_start, int64_t* o_end, int64_t* o_res,
                         int64_t* o_pay, int32_t* bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t x = pa[i], y = pb[i];
        const int64_t k = a_key[x], s = a_start[x];
        if (b_key[y] != k || b_start[y] != s) atomicOr(bad, 1);
        const int64_t seq = b_res[y];
        const int64_t rel = seq - log_base;
        int64_t pay = 0;
        if (rel < 0 || rel >= log_cap) atomicOr(bad, 2);
        else pay = log[seq % log_cap];
        o_key[i] = k;
        o_start[i] = s;
        o_end[i] = a_end[x];
        o_res[i] = a_res[x];
        o_pay[i] = pay;
    }
}

__global__ void k_fe_gather_log(const int64_t* log, int64_t cap, const int64_t* seq, int64_t n, int64_t* out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = log[seq[i] % cap];
}

// Copy the live log [base, end) from a ring of ocap words into a ring of ncap words.
__global__ void k_fe_recopy(const int64_t* o, int64_t ocap, int64_t* d, int64_t ncap, int64_t base, int64_t end) {
    for (int64_t q = base + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < end; q += (int64_t)gridDim.x * blockDim.x)
        d[q % ncap] = o[q % ocap];
}

static unsigned grid_n(int64_t n) {
    int64_t g = (n + 255) / 256;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 4096));
}

hipError_t fe_log_gather(const int64_t* log, int64_t cap, const int64_t* seq, int64_t n, int64_t* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fe_gather_log, dim3(grid_n(n)), dim3(256), 0, s, log, cap, seq, n, out);
    return hipGetLastError();
}

size_t fe_join_scratch_bytes(int64_t n) {
    size_t bytes = 0;
    rocprim::double_buffer<int64_t> kb(nullptr, nullptr);
    rocprim::double_buffer<uint32_t> vb(nullptr, nullptr);
    rocprim::radix_sort_pairs(nullptr, bytes, kb, vb, (size_t)std::max<int64_t>(n, 1));
    const size_t a = (size_t)std::max<int64_t>(n, 1);
    // sort temp + 2 key buffers (8 B) + 2 index buffers (4 B) per side, two sides
    return ((bytes + 255) / 256 * 256) + 2 * (a * 16 + a * 8) + 1024;
}

// (key, start) order of one side: indices sorted by start, then stably by key.
static hipError_t sort_side(int64_t n, const int64_t* key, const int64_t* start, uint32_t*& order, uint8_t*& p,
                            void* tmp, size_t tmp_bytes, hipStream_t s) {
    const size_t a = (size_t)n;
    int64_t* k0 = (int64_t*)p; p += a * 8;
    int64_t* k1 = (int64_t*)p; p += a * 8;
    uint32_t* v0 = (uint32_t*)p; p += a * 4;
    uint32_t* v1 = (uint32_t*)p; p += a * 4;
    hipLaunchKernelGGL(k_fe_iota32, dim3(grid_n(n)), dim3(256), 0, s, v0, n);
    hipError_t e = hipMemcpyAsync(k0, start, a * 8, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess) return e;
    rocprim::double_buffer<int64_t> kb(k0, k1);
    rocprim::double_buffer<uint32_t> vb(v0, v1);
    size_t bytes = tmp_bytes;
    if ((e = rocprim::radix_sort_pairs(tmp, bytes, kb, vb, a, 0, 64, s)) != hipSuccess) return e;
    // second pass: the keys of the start-sorted order, sorted stably
    int64_t* kk = kb.alternate();
    hipLaunchKernelGGL(k_fe_gather_key, dim3(grid_n(n)), dim3(256), 0, s, key, vb.current(), kk, n);
    rocprim::double_buffer<int64_t> kb2(kk, kb.current());
    rocprim::double_buffer<uint32_t> vb2(vb.current(), vb.alternate());
    bytes = tmp_bytes;
    if ((e = rocprim::radix_sort_pairs(tmp, bytes, kb2, vb2, a, 0, 64, s)) != hipSuccess) return e;
    order = vb2.current();
    return hipGetLastError();
}

hipError_t fe_join(int64_t n, const int64_t* a_key, const int64_t* a_start, const int64_t* a_end,
                   const int64_t* a_res, const int64_t* b_key, const int64_t* b_start, const int64_t* b_res,
                   const int64_t* log, int64_t log_base, int64_t log_cap, int64_t* o_key, int64_t* o_start,
                   int64_t* o_end, int64_t* o_res, int64_t* o_pay, void* scratch, size_t scratch_bytes,
                   int32_t* d_bad, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    size_t tmp_bytes = 0;
    {
        rocprim::double_buffer<int64_t> kb(nullptr, nullptr);
        rocprim::double_buffer<uint32_t> vb(nullptr, nullptr);
        rocprim::radix_sort_pairs(nullptr, tmp_bytes, kb, vb, (size_t)n);
    }
    if (scratch_bytes < fe_join_scratch_bytes(n)) return hipErrorInvalidValue;
    uint8_t* p = (uint8_t*)scratch;
    void* tmp = p;
    p += (tmp_bytes + 255) / 256 * 256;
    uint32_t *pa = nullptr, *pb = nullptr;
    hipError_t e = sort_side(n, a_key, a_start, pa, p, tmp, tmp_bytes, s);
    if (e == hipSuccess) e = sort_side(n, b_key, b_start, pb, p, tmp, tmp_bytes, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fe_zip, dim3(grid_n(n)), dim3(256), 0, s, n, pa, pb, a_key, a_start, a_end, a_res, b_key,
                       b_start, b_res, log, log_base, log_cap, o_key, o_start, o_end, o_res, o_pay, d_bad);
    return hipGetLastError();
}

hipError_t fe_iota64(int64_t* d, int64_t n, int64_t base, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_fe_iota64, dim3(grid_n(n)), dim3(256), 0, s, d, n, base);
    return hipGetLastError();
}

hipError_t fe_max_ts(const int64_t* ts, int64_t n, int64_t* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1024));
    hipLaunchKernelGGL(k_fe_max, dim3(g), dim3(256), 0, s, ts, n, out);
    return hipGetLastError();
}

hipError_t fe_log_regrow(const int64_t* o, int64_t ocap, int64_t* d, int64_t ncap, int64_t base, int64_t end,
                         hipStream_t s) {
    if (end <= base) return hipSuccess;
    hipLaunchKernelGGL(k_fe_recopy, dim3(grid_n(end - base)), dim3(256), 0, s, o, ocap, d, ncap, base, end);
    return hipGetLastError();
}

hipError_t fe_log_append(int64_t* log, int64_t cap, int64_t pos, const int64_t* src, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t at = pos % cap, n1 = std::min(n, cap - at);  // up to the ring's end, then from 0
    hipLaunchKernelGGL(k_fe_append, dim3(grid_n(n1)), dim3(256), 0, s, log, at, src, n1);
    if (n > n1) hipLaunchKernelGGL(k_fe_append, dim3(grid_n(n - n1)), dim3(256), 0, s, log, (int64_t)0, src + n1, n - n1);
    return hipGetLastError();
}

}  // namespace gw
