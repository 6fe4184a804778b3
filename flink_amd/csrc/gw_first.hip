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


#include "gw_first.h"
#include "gw_sort.h"

namespace gw {

__global__ void k_fe_iota64(int64_t* d, int64_t n, int64_t base) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        d[i] = base + i;
}

// int64 -> its unsigned radix order (sign bit flipped) less the column's smallest such value,
// gathered through idx (or not: idx null)
__global__ void k_fe_gather_key(const int64_t* src, const uint32_t* idx, uint64_t* dst, int64_t n, uint64_t lo) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = ((uint64_t)src[idx ? idx[i] : i] ^ 0x8000000000000000ull) - lo;
}

// Smallest and largest radix-order value of four columns (the join's keys and starts):
// out[2c] = min, out[2c + 1] = max of column c; out preset to (~0, 0).  The sorts then cover
// only the bits of max - min (keys below 2^24: 3 passes, not 8; one window start: none).
__global__ void __launch_bounds__(256) k_fe_range(const int64_t* c0, const int64_t* c1, const int64_t* c2,
                                                  const int64_t* c3, int64_t n, unsigned long long* out) {
    const int64_t* col[4] = {c0, c1, c2, c3};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        unsigned long long lo = ~0ull, hi = 0;
        for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
            const unsigned long long v = (unsigned long long)col[c][i] ^ 0x8000000000000000ull;
            lo = min(lo, v);
            hi = max(hi, v);
        }
        for (int o = 32; o > 0; o >>= 1) {
            lo = min(lo, (unsigned long long)__shfl_xor(lo, o));
            hi = max(hi, (unsigned long long)__shfl_xor(hi, o));
        }
        if (__lane_id() == 0) {
            atomicMin(&out[2 * c], lo);
            atomicMax(&out[2 * c + 1], hi);
        }
    }
}

__global__ void k_fe_range_init(unsigned long long* out) {
    if (threadIdx.x < 8) out[threadIdx.x] = (threadIdx.x & 1) ? 0ull : ~0ull;
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
    const size_t bytes = (size_t)sort_scratch_bytes(std::max<int64_t>(n, 1));
    const size_t a = (size_t)std::max<int64_t>(n, 1);
    // sort temp + 2 key buffers (8 B) + 2 index buffers (4 B) per side, two sides, the ranges
    return ((bytes + 255) / 256 * 256) + 2 * (a * 16 + a * 8) + 1024 + 64;
}

static int range_bits(uint64_t lo, uint64_t hi) {
    if (hi <= lo) return 0;
    return 64 - __builtin_clzll(hi - lo);
}

// (key, start) order of one side: indices sorted by start, then stably by key (gw_sort.hip,
// int64 values in radix order: the sign bit flipped, less the column's minimum; only the bits of
// the column's range are sorted).
static hipError_t sort_side(int64_t n, const int64_t* key, const int64_t* start, const uint64_t* rk,
                            const uint64_t* rs, uint32_t*& order, uint8_t*& p, void* tmp, hipStream_t s) {
    const size_t a = (size_t)n;
    uint64_t* k0 = (uint64_t*)p; p += a * 8;
    uint64_t* k1 = (uint64_t*)p; p += a * 8;
    uint32_t* v0 = (uint32_t*)p; p += a * 4;
    uint32_t* v1 = (uint32_t*)p; p += a * 4;
    const int sbits = range_bits(rs[0], rs[1]), kbits = range_bits(rk[0], rk[1]);
    int alt = 0;
    hipError_t e;
    if (sbits) hipLaunchKernelGGL(k_fe_gather_key, dim3(grid_n(n)), dim3(256), 0, s, start, (const uint32_t*)nullptr, k0, n,
                                  rs[0]);
    if ((e = sort_pairs_u64(k0, v0, k1, v1, n, 0, sbits, tmp, s, &alt, /*iota=*/true)) != hipSuccess) return e;
    uint32_t* va = alt ? v1 : v0;
    uint32_t* vb = alt ? v0 : v1;
    // second sort: the keys of the start-sorted order, stably
    uint64_t* kk = alt ? k0 : k1;
    uint64_t* ko = alt ? k1 : k0;
    if (!kbits) {
        order = va;
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_fe_gather_key, dim3(grid_n(n)), dim3(256), 0, s, key, va, kk, n, rk[0]);
    if ((e = sort_pairs_u64(kk, va, ko, vb, n, 0, kbits, tmp, s, &alt)) != hipSuccess) return e;
    order = alt ? vb : va;
    return hipGetLastError();
}

hipError_t fe_join(int64_t n, const int64_t* a_key, const int64_t* a_start, const int64_t* a_end,
                   const int64_t* a_res, const int64_t* b_key, const int64_t* b_start, const int64_t* b_res,
                   const int64_t* log, int64_t log_base, int64_t log_cap, int64_t* o_key, int64_t* o_start,
                   int64_t* o_end, int64_t* o_res, int64_t* o_pay, void* scratch, size_t scratch_bytes,
                   int32_t* d_bad, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const size_t tmp_bytes = (size_t)sort_scratch_bytes(n);
    if (scratch_bytes < fe_join_scratch_bytes(n)) return hipErrorInvalidValue;
    uint8_t* p = (uint8_t*)scratch;
    void* tmp = p;
    p += (tmp_bytes + 255) / 256 * 256;
    unsigned long long* d_range = (unsigned long long*)(p + 2 * ((size_t)n * 16 + (size_t)n * 8) + 1024);
    // the columns' ranges (one small device-to-host copy: the sorts' pass counts depend on it)
    hipLaunchKernelGGL(k_fe_range_init, dim3(1), dim3(64), 0, s, d_range);
    const unsigned rg = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 512));
    hipLaunchKernelGGL(k_fe_range, dim3(rg), dim3(256), 0, s, a_key, a_start, b_key, b_start, n, d_range);
    uint64_t r[8];
    hipError_t e = hipMemcpyAsync(r, d_range, sizeof r, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    // one range per column over both sides: equal (key, start) pairs map to equal sort keys
    uint64_t rk[2] = {std::min(r[0], r[4]), std::max(r[1], r[5])}, rs[2] = {std::min(r[2], r[6]), std::max(r[3], r[7])};
    uint32_t *pa = nullptr, *pb = nullptr;
    e = sort_side(n, a_key, a_start, rk, rs, pa, p, tmp, s);
    if (e == hipSuccess) e = sort_side(n, b_key, b_start, rk, rs, pb, p, tmp, s);
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
    // the live range as the few runs that are contiguous in both rings (device-to-device copies;
    // the element-wise k_fe_recopy did two 64-bit modulos per word: ~440 us per column of a
    // growing maxBy log, profiles/r6/maxby/)
    for (int64_t q = base; q < end;) {
        const int64_t oa = q % ocap, na = q % ncap;
        const int64_t len = std::min(end - q, std::min(ocap - oa, ncap - na));
        const hipError_t e = hipMemcpyAsync(d + na, o + oa, (size_t)len * 8, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
        q += len;
    }
    return hipSuccess;
}

hipError_t fe_log_append(int64_t* log, int64_t cap, int64_t pos, const int64_t* src, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t at = pos % cap, n1 = std::min(n, cap - at);  // up to the ring's end, then from 0
    hipLaunchKernelGGL(k_fe_append, dim3(grid_n(n1)), dim3(256), 0, s, log, at, src, n1);
    if (n > n1) hipLaunchKernelGGL(k_fe_append, dim3(grid_n(n - n1)), dim3(256), 0, s, log, (int64_t)0, src + n1, n - n1);
    return hipGetLastError();
}

// ---- minBy / maxBy (GW_FLAG_BY_FIELD) ----------------------------------------------------
// WindowedStream.minBy / maxBy (WindowedStream.java:725-771) reduce with ComparableAggregator's
// byAggregate branch (ComparableAggregator.java:88-95, Min/MaxByComparator in Comparator.java):
// the window's state is the ELEMENT whose field is the window's minimum / maximum, the first of
// equal ones in arrival order (first = true) or the last.  kids[0] folds MIN / MAX of the field
// (the row's result); at a fire one pass over the live log -- (payload, key, ts, field) of every
// record whose windows are not all cleaned -- picks the element: each record probes the fired
// rows of its windows in an open-addressing table of (key, start) and, when its field equals the
// row's result, offers its sequence (atomicMin for the first, atomicMax for the last).  A record
// is in a fired window's state exactly when it is in the log with a timestamp in the window: a
// record of a cleaned window is dropped, and a cleaned window never fires again.  For the first
// element this also holds for a lateness re-firing's prefix state (the earliest equal record
// precedes the late record that fired it).  Restored elements (sequences below `restored_end`)
// stand for their own window only: their timestamp is that window's start.

__device__ __forceinline__ uint64_t by_hash(int64_t key, int64_t start) {
    uint64_t x = (uint64_t)key * 0x9e3779b97f4a7c15ull ^ ((uint64_t)start + 0x632be59bd9b4e019ull) * 0xbf58476d1ce4e5b9ull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ int64_t by_floor_div(int64_t a, int64_t b) {
    const int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

// Field equality as Long.compareTo / Double.compare == 0 (NaNs equal, -0.0 != 0.0).
__device__ __forceinline__ bool by_equal(int64_t a, int64_t b, bool f64) {
    if (!f64) return a == b;
    const uint64_t qn = 0x7ff8000000000000ull;
    const bool na = ((uint64_t)a & 0x7fffffffffffffffull) > 0x7ff0000000000000ull;
    const bool nb = ((uint64_t)b & 0x7fffffffffffffffull) > 0x7ff0000000000000ull;
    return (na ? qn : (uint64_t)a) == (nb ? qn : (uint64_t)b);
}

__global__ void k_by_km_init(int64_t* km, int64_t* bound, int64_t nbk, int64_t init) {
    if (blockIdx.x == 0 && threadIdx.x == 0) { km[0] = INT64_MAX; km[1] = INT64_MIN; }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nbk; i += (int64_t)gridDim.x * blockDim.x)
        bound[i] = init;
}

// A field as an int64 in Double.compare / Long.compareTo order, equal exactly when by_equal says
// so (NaNs one value, -0.0 below 0.0).
__device__ __forceinline__ int64_t by_ord(int64_t v, bool f64) {
    if (!f64) return v;
    if (((uint64_t)v & 0x7fffffffffffffffull) > 0x7ff0000000000000ull) v = 0x7ff8000000000000ll;
    return v >= 0 ? v : v ^ 0x7fffffffffffffffll;
}

// floor((a) / b) for b > 0 by a double estimate corrected by one step each way (exact while
// |a| < 2^52; the integer division beyond): the scan runs it twice per log record.
__device__ __forceinline__ int64_t by_fdiv(int64_t a, int64_t b) {
    if (a > (1ll << 52) || a < -(1ll << 52)) return by_floor_div(a, b);
    int64_t q = (int64_t)floor((double)a / (double)b);
    if (q * b > a) --q;
    else if ((q + 1) * b <= a) ++q;
    return q;
}

// Rows into the table (one slot per row, duplicates included); sel[i] = the neutral sequence;
// km = [min, max] window index over the rows; bound[bucket] = the least (is_max) / greatest
// field order of the rows in the bucket (the top bits of the row's hash): a log record whose
// field lies beyond its bucket's bound equals no row there and skips the probe.
__global__ void k_by_build(int64_t n, const int64_t* key, const int64_t* start, const int64_t* res, int32_t* table,
                           uint64_t mask, int64_t* sel, int64_t init, int64_t offset, int64_t slide, int64_t* km,
                           int64_t* bound, int bk_shift, int is_max, int f64) {
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        sel[i] = init;
        const int64_t k = by_floor_div(start[i] - offset, slide);
        lo = min(lo, k);
        hi = max(hi, k);
        const uint64_t hh = by_hash(key[i], start[i]);
        const int64_t o = by_ord(res[i], f64 != 0);
        if (is_max) atomicMin((long long*)&bound[hh >> bk_shift], (long long)o);
        else atomicMax((long long*)&bound[hh >> bk_shift], (long long)o);
        uint64_t h = hh & mask;
        while (atomicCAS(&table[h], -1, (int32_t)i) != -1) h = (h + 1) & mask;
    }
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, (int64_t)__shfl_xor(lo, o));
        hi = max(hi, (int64_t)__shfl_xor(hi, o));
    }
    if (__lane_id() == 0 && lo <= hi) {
        atomicMin((long long*)&km[0], (long long)lo);
        atomicMax((long long*)&km[1], (long long)hi);
    }
}

struct ByScanArgs {
    const int64_t* log;  // 4 columns of cap words: payload, key, ts, field
    int64_t cap, lo, hi, restored_end;
    const int32_t* table;
    uint64_t mask;
    const int64_t *key, *start, *res;
    int64_t* sel;
    const int64_t* km;
    const int64_t* bound;
    int bk_shift, is_max;
    int64_t offset, slide, size;
    int last, f64;
};

__global__ void __launch_bounds__(256) k_by_scan(ByScanArgs a) {
    const int64_t k_lo = a.km[0], k_hi = a.km[1];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t q = a.lo + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int64_t at = q % a.cap;  // the ring position, advanced with q (no division per record)
    const int64_t step = stride % a.cap;
    for (; q < a.hi; q += stride) {
        const int64_t key = a.log[a.cap + at], ts = a.log[2 * a.cap + at], v = a.log[3 * a.cap + at];
        at += step;
        if (at >= a.cap) at -= a.cap;
        const int64_t vo = by_ord(v, a.f64 != 0);
        const int64_t kt = by_fdiv(ts - a.offset, a.slide);
        int64_t k0 = q < a.restored_end ? kt : by_fdiv(ts - a.offset - a.size, a.slide) + 1;
        const int64_t k1 = min(kt, k_hi);
        k0 = max(k0, k_lo);
        for (int64_t k = k0; k <= k1; ++k) {
            const int64_t s = a.offset + k * a.slide;
            const uint64_t hh = by_hash(key, s);
            const int64_t bd = a.bound[hh >> a.bk_shift];
            if (a.is_max ? vo < bd : vo > bd) continue;  // below every row's MAX in the bucket (above every MIN)
            uint64_t h = hh & a.mask;
            for (int32_t r; (r = a.table[h]) >= 0; h = (h + 1) & a.mask) {
                if (a.key[r] != key || a.start[r] != s || !by_equal(v, a.res[r], a.f64)) continue;
                if (a.last) atomicMax((long long*)&a.sel[r], (long long)q);
                else atomicMin((long long*)&a.sel[r], (long long)q);
            }
        }
    }
}

// o_pay[i] = the payload of row i's element; bad |= 2 when it is not in the log.
__global__ void k_by_emit(int64_t n, const int64_t* sel, const int64_t* log, int64_t cap, int64_t base, int64_t end,
                          int64_t* o_seq, int64_t* o_pay, int32_t* bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = sel[i];
        int64_t pay = 0;
        if (q < base || q >= end) atomicOr(bad, 2);
        else pay = log[q % cap];
        if (o_seq) o_seq[i] = q;
        if (o_pay) o_pay[i] = pay;
    }
}

// Buckets of the scan's filter: ~16 rows each (a power of two, the top bits of the row hash).
static int by_bucket_bits(int64_t n) {
    int b = 6;
    while (b < 30 && ((int64_t)1 << b) * 16 < n) ++b;
    return b;
}

size_t fe_by_scratch_bytes(int64_t n) {
    uint64_t tcap = 1024;
    while (tcap < (uint64_t)(2 * n)) tcap <<= 1;
    return tcap * 4 + (size_t)std::max<int64_t>(n, 1) * 8 + 256 + ((size_t)8 << by_bucket_bits(n));
}

hipError_t fe_by_select(int64_t n, const int64_t* key, const int64_t* start, const int64_t* res, const int64_t* log,
                        int64_t log_cap, int64_t log_base, int64_t log_end, int64_t restored_end, int64_t offset,
                        int64_t slide, int64_t size, bool last, bool f64, bool is_max, int64_t* o_seq,
                        int64_t* o_pay, void* scratch, size_t scratch_bytes, int32_t* d_bad, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (scratch_bytes < fe_by_scratch_bytes(n) || slide <= 0) return hipErrorInvalidValue;
    uint64_t tcap = 1024;
    while (tcap < (uint64_t)(2 * n)) tcap <<= 1;
    uint8_t* p = (uint8_t*)scratch;
    int64_t* km = (int64_t*)p;
    int64_t* sel = (int64_t*)(p + 256);
    int32_t* table = (int32_t*)(p + 256 + (size_t)n * 8);
    const int bbits = by_bucket_bits(n);
    const int64_t nbk = (int64_t)1 << bbits;
    int64_t* bound = (int64_t*)(p + 256 + (size_t)n * 8 + tcap * 4);
    hipError_t e = hipMemsetAsync(table, 0xff, tcap * 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_by_km_init, dim3(grid_n(nbk)), dim3(256), 0, s, km, bound, nbk,
                       is_max ? INT64_MAX : INT64_MIN);
    hipLaunchKernelGGL(k_by_build, dim3(grid_n(n)), dim3(256), 0, s, n, key, start, res, table, tcap - 1, sel,
                       last ? INT64_MIN : INT64_MAX, offset, slide, km, bound, 64 - bbits, is_max ? 1 : 0,
                       f64 ? 1 : 0);
    if (log_end > log_base) {
        ByScanArgs a{};
        a.log = log; a.cap = log_cap; a.lo = log_base; a.hi = log_end; a.restored_end = restored_end;
        a.table = table; a.mask = tcap - 1;
        a.bound = bound; a.bk_shift = 64 - bbits; a.is_max = is_max ? 1 : 0;
        a.key = key; a.start = start; a.res = res; a.sel = sel; a.km = km;
        a.offset = offset; a.slide = slide; a.size = size;
        a.last = last; a.f64 = f64;
        const int64_t m = log_end - log_base;
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((m + 255) / 256, 8192));
        hipLaunchKernelGGL(k_by_scan, dim3(g), dim3(256), 0, s, a);
    }
    hipLaunchKernelGGL(k_by_emit, dim3(grid_n(n)), dim3(256), 0, s, n, sel, log, log_cap, log_base, log_end, o_seq,
                       o_pay, d_bad);
    return hipGetLastError();
}

}  // namespace gw
