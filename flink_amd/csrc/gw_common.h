// gw_common.h — shared by the gfx950 kernels and the host runtime of libgpuwin.so.
//
// Semantics restated here (cited per function) are those of the reference's
// keyed event-time window path; the state layout is this library's own
// MI355X-first design: an open-addressing table of per-key slots in
// HBM, each slot holding a ring of pane (slice) accumulators.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpuwin.h"

#define GW_HD __host__ __device__ __forceinline__

namespace gw {

constexpr int64_t kEmptyKey = INT64_MIN;  // slot sentinel; the real key INT64_MIN lives in slot `cap`
constexpr int kMaxRing = 64;              // pane ring length limit (64-bit presence mask)
constexpr int kMaxProbe = 128;            // linear-probe limit before a record is parked

// ---------------------------------------------------------------------------
// Packed exchange records (include/gpuwin.h gw_pack_geom; gw_keygroups.hip partition,
// gw_exchange.cpp): one 8-byte word instead of 24 B of key, ts and value,
//   lo32 = key, hi32 = value << 4 | d   (d = the record's pane - base_pane, 0 <= d < 16)
// for a record whose key is in [0, 2^32), whose value (when the batch has values) is in
// [-2^27, 2^27), and whose pane floor((ts - offset) / pane) lies in [base_pane, base_pane + 16).
// Unpacked, its timestamp is its pane's start: for tumbling / sliding windows with
// size >= slide and pane = gcd(size, slide) every window decision (assignWindows, isLate,
// the cleanup time) depends on the pane alone.
// ---------------------------------------------------------------------------
using PackGeom = gw_pack_geom;
constexpr int kPackPanes = 16;
constexpr int64_t kPackValLimit = 1ll << 27;

GW_HD bool pack_word(const PackGeom& g, int64_t key, int64_t ts, bool has_val, int64_t v, uint64_t& w) {
    if ((uint64_t)key >> 32) return false;
    constexpr int64_t kLim = 1ll << 62;  // |ts|, |offset| below it: no overflow below
    if (ts < -kLim || ts >= kLim || g.offset < -kLim || g.offset >= kLim) return false;
    const int64_t rel = ts - g.offset;
    int64_t d, b0, r, lim;
    if (!__builtin_mul_overflow(g.base_pane, g.pane, &b0) && !__builtin_mul_overflow(g.pane, (int64_t)kPackPanes, &lim) &&
        !__builtin_sub_overflow(rel, b0, &r)) {
        // floor(rel / pane) - base_pane in [0, 16)  <=>  0 <= rel - base_pane * pane < 16 * pane;
        // the pane offset then by four compares (no 64-bit division: ~100 instructions per
        // record on the GPU, where this runs once per exchanged record)
        if (r < 0 || r >= lim) return false;
        d = r >= 8 * g.pane ? 8 : 0;
        if (r >= (d + 4) * g.pane) d += 4;
        if (r >= (d + 2) * g.pane) d += 2;
        if (r >= (d + 1) * g.pane) d += 1;
    } else {
        int64_t q = rel / g.pane;
        if (rel % g.pane < 0) --q;  // floor (TimeWindow.getWindowStartWithOffset)
        if (__builtin_sub_overflow(q, g.base_pane, &d) || d < 0 || d >= kPackPanes) return false;
    }
    if (!has_val) v = 0;
    else if (v < -kPackValLimit || v >= kPackValLimit) return false;
    w = (uint64_t)(uint32_t)key | ((uint64_t)(((uint32_t)(int32_t)v << 4) | (uint32_t)d) << 32);
    return true;
}
GW_HD void unpack_word(const PackGeom& g, uint64_t w, int64_t& key, int64_t& ts, int64_t& v) {
    const uint32_t hi = (uint32_t)(w >> 32);
    key = (int64_t)(uint32_t)w;
    ts = (g.base_pane + (int64_t)(hi & 15u)) * g.pane + g.offset;
    v = (int64_t)((int32_t)hi >> 4);
}

// ---------------------------------------------------------------------------
// Java hashing (bit-exact with the reference)
// ---------------------------------------------------------------------------
GW_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// MathUtils.bitMix (flink-core/.../util/MathUtils.java:194-201)
GW_HD int32_t bit_mix(int32_t in) {
    uint32_t h = (uint32_t)in;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return (int32_t)h;
}

// MathUtils.murmurHash(int) (MathUtils.java:137-155)
GW_HD int32_t murmur_hash(int32_t code) {
    uint32_t c = (uint32_t)code;
    c *= 0xcc9e2d51u;
    c = rotl32(c, 15);
    c *= 0x1b873593u;
    c = rotl32(c, 13);
    c = c * 5u + 0xe6546b64u;
    c ^= 4u;
    int32_t r = bit_mix((int32_t)c);
    if (r >= 0) return r;
    if (r != INT32_MIN) return -r;
    return 0;
}

// JDK Long.hashCode
GW_HD int32_t java_long_hash(int64_t v) {
    uint64_t u = (uint64_t)v;
    return (int32_t)(uint32_t)(u ^ (u >> 32));
}

// KeyGroupRangeAssignment.computeKeyGroupForKeyHash (:75-77)
GW_HD int32_t key_group_for_hash(int32_t h, int32_t max_p) { return murmur_hash(h) % max_p; }
// KeyGroupRangeAssignment.computeOperatorIndexForKeyGroup (:124-127)
GW_HD int32_t operator_for_key_group(int32_t max_p, int32_t p, int32_t kg) { return kg * p / max_p; }

// State-table hash (this library's own; independent of the key-group hash so that
// the slots of one key group are spread over the whole table): a multiply by the 64-bit
// golden ratio (the region is the product's top bits, Fibonacci hashing), then an xor-shift
// that folds the top half into the bottom one (the home slot is the low bits).  Both steps
// are bijections; one 64-bit multiply instead of the murmur finalizer's two, since every
// region-path record hashes in each pass.
GW_HD uint64_t slot_hash(int64_t key) {
    uint64_t x = (uint64_t)key * 0x9e3779b97f4a7c15ull;
    return x ^ (x >> 32);
}
// Its inverse: the xor-shift by 32 is self-inverse, the multiplier odd.  The compact
// region-path records carry the hash and the apply recovers the key from it.
GW_HD int64_t slot_unhash(uint64_t x) {
    x ^= x >> 32;
    return (int64_t)(x * 0xf1de83e19937733dull);  // 0x9e3779b97f4a7c15^-1 mod 2^64
}

// ---------------------------------------------------------------------------
// Double ordering (Double.compare: NaN largest and canonical, -0.0 < 0.0) as a
// signed int64 order, so min/max run as integer atomics.
// ---------------------------------------------------------------------------
GW_HD int64_t f64_order_key(int64_t bits) {
    if (((bits >> 52) & 0x7ff) == 0x7ff && (bits & 0xfffffffffffffLL)) bits = 0x7ff8000000000000LL;
    return bits ^ ((bits >> 63) & 0x7fffffffffffffffLL);
}
GW_HD int64_t f64_from_order_key(int64_t k) { return k ^ ((k >> 63) & 0x7fffffffffffffffLL); }

GW_HD double bits_to_f64(int64_t b) { return __builtin_bit_cast(double, b); }
GW_HD int64_t f64_to_bits(double d) { return __builtin_bit_cast(int64_t, d); }

// ---------------------------------------------------------------------------
// Accumulator cells (one per (key, pane)).  Two 8-byte words; word 1 is only
// used by AVG.  Identity values make "merge into an empty cell" a plain RMW.
// ---------------------------------------------------------------------------
GW_HD int cell_words(int agg) { return (agg == GW_AVG_I64 || agg == GW_AVG_F64) ? 2 : 1; }
GW_HD bool result_is_double(int agg) {
    return agg == GW_SUM_F64 || agg == GW_MIN_F64 || agg == GW_MAX_F64 || agg == GW_AVG_I64 ||
           agg == GW_AVG_F64;
}
GW_HD int64_t identity0(int agg) {
    switch (agg) {
    case GW_SUM_F64: return (int64_t)0x8000000000000000ull;  // -0.0: x + (-0.0) == x for all x
    case GW_MIN_I64: case GW_MIN_F64: return INT64_MAX;
    case GW_MAX_I64: case GW_MAX_F64: return INT64_MIN;
    default: return 0;  // COUNT, SUM_I64, SUM_I32, AVG_*(sum; +0.0 for AVG_F64)
    }
}
// The accumulator contribution of a single raw record value.
GW_HD void record_cell(int agg, int64_t v, int64_t& a0, int64_t& a1) {
    a1 = 1;
    switch (agg) {
    case GW_COUNT: a0 = 1; break;
    case GW_MIN_F64: case GW_MAX_F64: a0 = f64_order_key(v); break;
    default: a0 = v; break;
    }
}
// Fold cell (b0,b1) into (a0,a1) on the host / in registers.
GW_HD void fold_cell(int agg, int64_t& a0, int64_t& a1, int64_t b0, int64_t b1) {
    switch (agg) {
    case GW_COUNT: case GW_SUM_I64: case GW_SUM_I32:
        a0 = (int64_t)((uint64_t)a0 + (uint64_t)b0); break;
    case GW_SUM_F64: a0 = f64_to_bits(bits_to_f64(a0) + bits_to_f64(b0)); break;
    case GW_MIN_I64: case GW_MIN_F64: a0 = a0 < b0 ? a0 : b0; break;
    case GW_MAX_I64: case GW_MAX_F64: a0 = a0 > b0 ? a0 : b0; break;
    case GW_AVG_I64:
        a0 = (int64_t)((uint64_t)a0 + (uint64_t)b0); a1 += b1; break;
    case GW_AVG_F64:
        a0 = f64_to_bits(bits_to_f64(a0) + bits_to_f64(b0)); a1 += b1; break;
    }
}
// Output column bits (int64 or IEEE double) — AggregateFunction.getResult / the
// reduced field of SumAggregator / ComparableAggregator.
GW_HD int64_t cell_result(int agg, int64_t a0, int64_t a1) {
    switch (agg) {
    case GW_SUM_I32: return (int64_t)(int32_t)(uint32_t)(uint64_t)a0;  // Java int wrap-around
    case GW_MIN_F64: case GW_MAX_F64: return f64_from_order_key(a0);
    case GW_AVG_I64: return f64_to_bits((double)a0 / (double)a1);
    case GW_AVG_F64: return f64_to_bits(bits_to_f64(a0) / (double)a1);
    default: return a0;
    }
}

// ---------------------------------------------------------------------------
// 64-bit unsigned division by a runtime-invariant divisor (Granlund-Montgomery
// round-up method): q = (t + ((n - t) >> 1)) >> (l - 1), t = mulhi(M, n).
// ---------------------------------------------------------------------------
struct UDiv64 {
    uint64_t magic;
    uint32_t shift;   // l - 1 (or 0 with is_pow2 handling)
    uint32_t mode;    // 0: general, 1: divisor == 1
};
GW_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
GW_HD uint64_t udiv64(uint64_t n, const UDiv64& d) {
    if (d.mode == 1) return n;
    uint64_t t = mulhi64(d.magic, n);
    return (t + ((n - t) >> 1)) >> d.shift;
}

}  // namespace gw
