// gw_pane.hip — gfx950 kernels of the tumbling / sliding (non-merging) window path.
//
// Reference semantics (paths relative to the Flink tree):
//   * window assignment: TumblingEventTimeWindows.assignWindows (RS/api/windowing/
//     assigners/TumblingEventTimeWindows.java:69-85), SlidingEventTimeWindows.assignWindows
//     (SlidingEventTimeWindows.java:77-90), TimeWindow.getWindowStartWithOffset
//     (RS/api/windowing/windows/TimeWindow.java:264-272)
//   * per-record state update: WindowOperator.processElement non-merging branch
//     (RS/runtime/operators/windowing/WindowOperator.java:405-433) -> HeapReducingState /
//     HeapAggregatingState.add (RR/state/heap/HeapReducingState.java:90-97,
//     HeapAggregatingState.java:94-102)
//   * lateness: WindowOperator.isWindowLate / isElementLate (:609-624)
//   * firing: EventTimeTrigger (RS/api/windowing/triggers/EventTimeTrigger.java:37-52) +
//     InternalTimerServiceImpl.tryAdvanceWatermark (RS/api/operators/
//     InternalTimerServiceImpl.java:328-347) + WindowOperator.onEventTime (:450-494):
//     with allowed lateness 0 the fired set at watermark wm is every (key, window) with
//     state and end-1 <= wm, each exactly once, then purged.
//
// MI355X design: instead of one state entry per (key, window) (Flink
// duplicates each record into size/slide windows, docs windows.md:1376), each key owns
// ONE slot holding a ring of R pane accumulators, pane width g = gcd(size, slide).  A
// record does one RMW into one pane; a window is the fold of its size/g panes at fire
// time.  Window boundaries are pane boundaries, so the fold equals the reference's
// per-window state for every associative aggregate of the closed set.
//
// Three ingest paths share the table (gw_kernels.h layout):
//   region  (large batches)  k_part_hist/cols/scatter (one or two LDS-sorted passes) ->
//           k_rgn_apply: records are bucketed by table region, one workgroup owns a
//           region, applies its records with LDS atomics on an LDS copy of the region's
//           keys / mask / active pane arrays, and writes them back coalesced.  No device
//           atomics on the state; every HBM access is a contiguous stream.
//   direct  (small batches)  k_ingest: one device-scope atomic per record.
//   preagg  (few keys)       k_ingest_preagg: LDS combine per (slot, pane), then atomics.
#include "gw_kernels.h"

#include <algorithm>

namespace gw {

template <int AGG>
__device__ __forceinline__ constexpr bool uses_mask() {
    return !(AGG == GW_COUNT || AGG == GW_AVG_I64 || AGG == GW_AVG_F64);
}

// Ring positions of a slot holding a non-null accumulator.  COUNT / AVG carry a count
// in the cell, so presence is `count != 0`; the others keep an explicit mask.
template <int AGG>
__device__ __forceinline__ uint64_t presence(const PaneTable& t, int64_t g) {
    if constexpr (uses_mask<AGG>()) {
        return pt_mask_get(t, g);
    } else {
        uint64_t m = 0;
        for (int r = 0; r < t.ring; ++r)
            if (pt_cell(t, g, r)[t.words - 1] != 0) m |= 1ull << r;
        return m;
    }
}
__device__ __forceinline__ uint64_t presence_rt(const PaneTable& t, int64_t g) {
    if (t.has_mask) return pt_mask_get(t, g);
    uint64_t m = 0;
    for (int r = 0; r < t.ring; ++r)
        if (pt_cell(t, g, r)[t.words - 1] != 0) m |= 1ull << r;
    return m;
}

// Per-record classification: late / parked (outside the pane ring) / in ring.
enum { REC_SKIP = 0, REC_RING = 1, REC_DEFER = 2 };
template <int AGG>
__device__ __forceinline__ int classify(const IngestArgs& a, int64_t ts, int64_t v, uint32_t& pos, int64_t& pane,
                                        int64_t& c0, int64_t& c1, unsigned long long& late,
                                        unsigned long long& flags) {
    if (ts == INT64_MIN) { flags |= GW_DF_NO_TS; return REC_SKIP; }
    if (ts < a.t_late) {
        if (a.late_exact) late++;
        else flags |= GW_DF_RANGE;
        return REC_SKIP;
    }
    const uint64_t R = (uint64_t)a.t.ring;
    const uint64_t q = udiv64((uint64_t)ts - (uint64_t)a.t_late, a.div);
    record_cell(AGG, v, c0, c1);
    pane = a.p_late + (int64_t)q;
    const uint64_t rel = q - a.delta;
    if (q >= a.delta && rel < R) {
        uint32_t p = (uint32_t)a.b_pos + (uint32_t)rel;
        if (p >= R) p -= (uint32_t)R;
        pos = p;
        return REC_RING;
    }
    if (q > (uint64_t)(INT64_MAX - a.p_late)) flags |= GW_DF_RANGE;
    return REC_DEFER;
}

template <int AGG>
__device__ __forceinline__ void mask_set(const PaneTable& t, int64_t g, uint32_t pos) {
    if constexpr (uses_mask<AGG>()) {
        mask_set_bit(pt_mask_base(t, g >> t.log2S), g & (pt_S(t) - 1), t.mask_shift, pos);
    }
}

__device__ __forceinline__ void defer_write(const IngestArgs& a, bool defer, int64_t key, int64_t pane, int64_t c0,
                                            int64_t c1) {
    const unsigned long long off = wave_reserve(&a.st->n_deferred, defer);
    if (defer) {
        a.d_key[off] = key;
        a.d_pane[off] = pane;
        a.d_a0[off] = c0;
        a.d_a1[off] = c1;
    }
}

template <int AGG>
__global__ void __launch_bounds__(256) k_table_init(PaneTable t) {
    const int64_t id0 = identity0(AGG);
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g <= t.cap; g += (int64_t)gridDim.x * blockDim.x) {
        *pt_key(t, g) = kEmptyKey;
        if (t.has_mask) pt_mask_put(t, g, 0);
        for (int r = 0; r < t.ring; ++r) {
            int64_t* c = pt_cell(t, g, r);
            c[0] = id0;
            if (t.words == 2) c[1] = 0;
        }
    }
}

// ---------------------------------------------------------------------------
// direct path
// ---------------------------------------------------------------------------
// Continue a region-local linear probe from home slot j (whose key was read as k0).
__device__ __forceinline__ int64_t pt_probe_from(const PaneTable& t, int64_t key, int64_t r, int64_t j, int64_t k0,
                                                 bool& inserted) {
    inserted = false;
    const int64_t S = pt_S(t);
    int64_t* keys = pt_region(t, r);
    int64_t k = k0;
    const int lim = S < kMaxProbe ? (int)S : kMaxProbe;
    for (int p = 0; p < lim; ++p) {
        int64_t* kp = keys + j;
        if (p) k = *(volatile int64_t*)kp;
        if (k == key) return (r << t.log2S) + j;
        if (k == kEmptyKey) {
            const unsigned long long prev = atomicCAS((unsigned long long*)kp, (unsigned long long)kEmptyKey,
                                                      (unsigned long long)key);
            if (prev == (unsigned long long)kEmptyKey) { inserted = true; return (r << t.log2S) + j; }
            if ((int64_t)prev == key) return (r << t.log2S) + j;
        }
        j = (j + 1) & (S - 1);
    }
    return -1;
}

// One device-scope atomic into the record's (slot, pane) cell (+ presence bit on first
// touch for SUM/MIN/MAX).  U records per thread issue their first probes together.
template <int AGG, int U>
__global__ void __launch_bounds__(256) k_ingest(IngestArgs a) {
    const int64_t tile = (int64_t)blockDim.x * U;
    const int64_t stride = (int64_t)gridDim.x * tile;
    unsigned long long late = 0, ins = 0, flags = 0, occ = 0;
    for (int64_t base = blockIdx.x * tile; base < a.n; base += stride) {
        int64_t key[U], c0[U], c1[U], pane[U], k0[U], reg[U], home[U];
        uint32_t pos[U];
        int state[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)u * blockDim.x + threadIdx.x;
            state[u] = REC_SKIP;
            key[u] = 0; c0[u] = 0; c1[u] = 0; pane[u] = 0; pos[u] = 0;
            if (i < a.n) {
                key[u] = a.key[i];
                state[u] = classify<AGG>(a, a.ts[i], a.val ? a.val[i] : 0, pos[u], pane[u], c0[u], c1[u], late,
                                         flags);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t h = slot_hash(key[u]);
            reg[u] = pt_key_region(a.t, h);
            home[u] = pt_home(a.t, h);
            k0[u] = (state[u] == REC_RING && key[u] != kEmptyKey)
                        ? *(volatile int64_t*)(pt_region(a.t, reg[u]) + home[u])
                        : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (state[u] != REC_RING) continue;
            int64_t g;
            if (key[u] == kEmptyKey) {
                g = a.t.cap;
            } else {
                bool inserted;
                g = pt_probe_from(a.t, key[u], reg[u], home[u], k0[u], inserted);
                ins += inserted;
            }
            if (g < 0) { flags |= GW_DF_TABLE_FULL; state[u] = REC_DEFER; continue; }
            cell_atomic<AGG>(pt_cell(a.t, g, pos[u]), c0[u], c1[u]);
            mask_set<AGG>(a.t, g, pos[u]);
            occ |= 1ull << pos[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) defer_write(a, state[u] == REC_DEFER, key[u], pane[u], c0[u], c1[u]);
    }
    block_commit(a.st, late, ins, flags, occ);
}

// ---------------------------------------------------------------------------
// LDS pre-aggregation path (low key cardinality per batch, e.g. YSB's 100 campaigns)
// ---------------------------------------------------------------------------
constexpr int kLdsCells = 2048;
constexpr int kPreaggItems = 8;

template <int AGG>
__device__ __forceinline__ void lds_cell_add(long long* a0, long long* a1, int64_t c0, int64_t c1) {
    if constexpr (AGG == GW_COUNT || AGG == GW_SUM_I64 || AGG == GW_SUM_I32) {
        atomicAdd((unsigned long long*)a0, (unsigned long long)c0);
    } else if constexpr (AGG == GW_SUM_F64) {
        atomicAdd((double*)a0, bits_to_f64(c0));
    } else if constexpr (AGG == GW_MIN_I64 || AGG == GW_MIN_F64) {
        atomicMin(a0, (long long)c0);
    } else if constexpr (AGG == GW_MAX_I64 || AGG == GW_MAX_F64) {
        atomicMax(a0, (long long)c0);
    } else if constexpr (AGG == GW_AVG_I64) {
        atomicAdd((unsigned long long*)a0, (unsigned long long)c0);
        atomicAdd((unsigned long long*)a1, (unsigned long long)c1);
    } else {
        atomicAdd((double*)a0, bits_to_f64(c0));
        atomicAdd((unsigned long long*)a1, (unsigned long long)c1);
    }
}

template <int AGG>
__global__ void __launch_bounds__(256) k_ingest_preagg(IngestArgs a) {
    constexpr bool AV = AGG == GW_AVG_I64 || AGG == GW_AVG_F64;
    __shared__ unsigned long long s_cell[kLdsCells];
    __shared__ long long s_a0[kLdsCells];
    __shared__ long long s_a1[AV ? kLdsCells : 1];
    const int64_t tile = (int64_t)blockDim.x * kPreaggItems;
    const uint64_t R = (uint64_t)a.t.ring;
    const int64_t id0 = identity0(AGG);
    unsigned long long late = 0, ins = 0, flags = 0, occ = 0, cells = 0;
    for (int64_t t0 = blockIdx.x * tile; t0 < a.n; t0 += (int64_t)gridDim.x * tile) {
        for (int j = threadIdx.x; j < kLdsCells; j += blockDim.x) {
            s_cell[j] = ~0ull;
            s_a0[j] = id0;
            if constexpr (AV) s_a1[j] = 0;
        }
        __syncthreads();
#pragma unroll 1
        for (int it = 0; it < kPreaggItems; ++it) {
            const int64_t i = t0 + (int64_t)it * blockDim.x + threadIdx.x;
            int state = REC_SKIP;
            int64_t key = 0, pane = 0, c0 = 0, c1 = 0;
            uint32_t pos = 0;
            if (i < a.n) {
                key = a.key[i];
                state = classify<AGG>(a, a.ts[i], a.val ? a.val[i] : 0, pos, pane, c0, c1, late, flags);
            }
            if (state == REC_RING) {
                bool inserted;
                const int64_t g = pt_find_or_insert(a.t, key, inserted);
                ins += inserted;
                if (g < 0) {
                    flags |= GW_DF_TABLE_FULL;
                    state = REC_DEFER;
                } else {
                    occ |= 1ull << pos;
                    const unsigned long long cell = (unsigned long long)(g * (int64_t)R + pos);
                    uint32_t h = (uint32_t)slot_hash((int64_t)cell) & (kLdsCells - 1);
                    bool done = false;
                    for (int p = 0; p < 32 && !done; ++p) {
                        unsigned long long cur = s_cell[h];
                        if (cur == ~0ull) cur = atomicCAS(&s_cell[h], ~0ull, cell);
                        if (cur == ~0ull || cur == cell) {
                            lds_cell_add<AGG>(&s_a0[h], &s_a1[AV ? h : 0], c0, c1);
                            done = true;
                        }
                        h = (h + 1) & (kLdsCells - 1);
                    }
                    if (!done) {  // LDS table saturated: straight to HBM
                        cell_atomic<AGG>(pt_cell(a.t, g, pos), c0, c1);
                        mask_set<AGG>(a.t, g, pos);
                    }
                }
            }
            defer_write(a, state == REC_DEFER, key, pane, c0, c1);
        }
        __syncthreads();
        for (int j = threadIdx.x; j < kLdsCells; j += blockDim.x) {
            const unsigned long long cellu = s_cell[j];
            if (cellu == ~0ull) continue;
            cells++;
            const int64_t cell = (int64_t)cellu;
            const int64_t g = cell / (int64_t)R;
            const uint32_t pos = (uint32_t)(cell - g * (int64_t)R);
            int64_t b1 = 0;
            if constexpr (AV) b1 = s_a1[j];
            cell_atomic<AGG>(pt_cell(a.t, g, pos), s_a0[j], b1);
            mask_set<AGG>(a.t, g, pos);
        }
        __syncthreads();
    }
    block_commit(a.st, late, ins, flags, occ, cells);
}

// ---------------------------------------------------------------------------
// region path
// ---------------------------------------------------------------------------
// In-ring records are bucketed by table region (the top log2nreg bits of the key
// hash) in at most two counting passes of <= 256 buckets each: pass 1 on
// the top d1 region bits, pass 2 on the remaining d2 bits inside each pass-1 bucket.
// Every pass sorts its 4096-record tile by bucket in LDS first and then writes each
// bucket's run with consecutive lanes, so all HBM writes are whole-line streams
// (single scattered 8-B stores turn into partial-line read-modify-writes in HBM3E and
// were measured at ~30 G stores/s).  k_rgn_apply then owns one region per workgroup.
constexpr int kPartThreads = 512;
constexpr int kPartItems = kPartTile / kPartThreads;

__device__ __forceinline__ int64_t rgn_of(const PaneTable& t, int64_t key) { return pt_key_region(t, slot_hash(key)); }

// Exclusive scan of h[0..nb) (nb <= 256) into out[]; executed by wave 0.
__device__ __forceinline__ void scan_buckets(const uint32_t* h, uint32_t* out, int nb) {
    if (threadIdx.x >= 64) return;
    const int l = threadIdx.x;
    uint32_t v[4], sum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        v[q] = 4 * l + q < nb ? h[4 * l + q] : 0u;
        sum += v[q];
    }
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t up = __shfl_up(incl, o);
        if (l >= o) incl += up;
    }
    uint32_t ex = incl - sum;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (4 * l + q < nb) out[4 * l + q] = ex;
        ex += v[q];
    }
}

// Pass-2 tile g -> its pass-1 bucket and record range (false: g beyond the last tile).
__device__ __forceinline__ bool pass2_tile(const IngestArgs& a, int64_t g, int& b1, int64_t& lo, int64_t& hi) {
    const int nb1 = 1 << a.d1_bits;
    if (g >= a.p2_tile0[nb1]) return false;
    int l = 0, h = nb1 - 1;  // last bucket with tile0 <= g
    while (l < h) {
        const int mid = (l + h + 1) >> 1;
        if (a.p2_tile0[mid] <= g) l = mid;
        else h = mid - 1;
    }
    b1 = l;
    lo = a.p1_base[l] + (g - a.p2_tile0[l]) * kPartTile;
    hi = min(a.p1_base[l + 1], lo + (int64_t)kPartTile);
    return true;
}

// Histogram of one tile: pass 1 over the input batch (classifying records), pass 2
// over one pass-1 bucket.  counts[g][b] (stride kPartBuckets).
template <int AGG, int PASS>
__global__ void __launch_bounds__(kPartThreads) k_part_hist(IngestArgs a) {
    __shared__ uint32_t lh[kPartBuckets];
    __shared__ unsigned long long s_occ;
    const int64_t g = blockIdx.x;
    int64_t lo, hi;
    int b1 = 0;
    if constexpr (PASS == 1) {
        lo = g * kPartTile;
        hi = min(a.n, lo + (int64_t)kPartTile);
    } else {
        if (!pass2_tile(a, g, b1, lo, hi)) return;
    }
    for (int b = threadIdx.x; b < kPartBuckets; b += blockDim.x) lh[b] = 0;
    if (threadIdx.x == 0) s_occ = 0;
    __syncthreads();
    unsigned long long late = 0, flags = 0, occ = 0;
    const int64_t m2 = ((int64_t)1 << a.d2_bits) - 1;
    // all of this thread's loads first (kPartItems in flight), then the LDS counts
    int64_t kk[kPartItems], tt[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = lo + it * kPartThreads + threadIdx.x;
        kk[it] = 0;
        tt[it] = INT64_MIN;
        if (i < hi) {
            if constexpr (PASS == 1) {
                kk[it] = a.key[i];
                tt[it] = a.ts[i];
            } else {
                kk[it] = a.p1_key[i];
            }
        }
    }
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = lo + it * kPartThreads + threadIdx.x;
        if (i >= hi) continue;
        if constexpr (PASS == 1) {
            uint32_t pos = 0;
            int64_t pane = 0, c0 = 0, c1 = 0;
            if (classify<AGG>(a, tt[it], 0, pos, pane, c0, c1, late, flags) == REC_RING && kk[it] != kEmptyKey) {
                atomicAdd(&lh[rgn_of(a.t, kk[it]) >> a.d2_bits], 1u);
                occ |= 1ull << pos;
            }
        } else {
            atomicAdd(&lh[rgn_of(a.t, kk[it]) & m2], 1u);
        }
    }
    if constexpr (PASS == 1) {  // one device atomic per block (same-address atomics serialise)
        occ = wave_ior(occ);
        if (__lane_id() == 0 && occ) atomicOr(&s_occ, occ);
    }
    __syncthreads();
    if (PASS == 1 && threadIdx.x == 0 && s_occ) atomicOr(a.batch_occ, s_occ);
    uint32_t* row = (PASS == 1 ? a.p_counts1 : a.p_counts2) + g * kPartBuckets;
    for (int b = threadIdx.x; b < kPartBuckets; b += blockDim.x) row[b] = lh[b];
}

// Pass-1 columns: for each bucket (one block) an exclusive scan over the tiles; the
// bucket total goes to base[b].
__global__ void __launch_bounds__(256) k_part_cols1(uint32_t* counts, int64_t tiles, int64_t* base) {
    __shared__ uint32_t part[256];
    const int b = blockIdx.x;
    uint32_t carry = 0;
    for (int64_t c = 0; c < tiles; c += 256) {
        const int64_t t = c + threadIdx.x;
        const uint32_t v = t < tiles ? counts[t * kPartBuckets + b] : 0u;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {
            const uint32_t x = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0u;
            __syncthreads();
            part[threadIdx.x] += x;
            __syncthreads();
        }
        if (t < tiles) counts[t * kPartBuckets + b] = carry + part[threadIdx.x] - v;
        carry += part[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) base[b] = carry;
}

// Exclusive scan of base[0..n) in place (one block); base[n] = total.  Pass 1 also
// lays out the pass-2 tiles: tile0[b] = first tile of bucket b, tile0[n] = tiles.
__global__ void __launch_bounds__(1024) k_rgn_bases(int64_t* base, int64_t n, int64_t* tile0) {
    __shared__ int64_t part[1024];
    const int64_t per = (n + blockDim.x - 1) / blockDim.x;
    const int64_t lo = threadIdx.x * per, hi = min(n, lo + per);
    for (int round = 0; round < (tile0 ? 2 : 1); ++round) {
        int64_t* arr = round ? tile0 : base;
        if (round) {  // tiles per bucket from the scanned bases
            for (int64_t i = lo; i < hi; ++i) tile0[i] = (base[i + 1] - base[i] + kPartTile - 1) / kPartTile;
        }
        int64_t s = 0;
        for (int64_t i = lo; i < hi; ++i) s += arr[i];
        part[threadIdx.x] = s;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const int64_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
            __syncthreads();
            part[threadIdx.x] += v;
            __syncthreads();
        }
        int64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t v = arr[i];
            arr[i] = run;
            run += v;
        }
        if (threadIdx.x == blockDim.x - 1) arr[n] = part[blockDim.x - 1];
        __syncthreads();
    }
}

// Pass-2 columns: one thread per region, exclusive scan over the tiles of its pass-1
// bucket; region totals to rg_base[r] (scanned next by k_rgn_bases).
__global__ void __launch_bounds__(256) k_part_cols2(IngestArgs a) {
    const int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (r >= a.t.nreg) return;
    const int64_t b1 = r >> a.d2_bits, s = r & (((int64_t)1 << a.d2_bits) - 1);
    uint32_t run = 0;
    for (int64_t g = a.p2_tile0[b1]; g < a.p2_tile0[b1 + 1]; ++g) {
        uint32_t* c = a.p_counts2 + g * kPartBuckets + s;
        const uint32_t v = *c;
        *c = run;
        run += v;
    }
    a.rg_base[r] = run;
}

// Scatter one tile: classify (pass 1), rank each record inside its bucket with an LDS
// atomic, place it in LDS in bucket order, then stream every bucket run out with
// consecutive lanes.  Pass 1 also handles late / parked / sentinel-key records.
template <int AGG, int PASS>
__global__ void __launch_bounds__(kPartThreads) k_part_scatter(IngestArgs a) {
    constexpr bool AV = AGG == GW_AVG_I64 || AGG == GW_AVG_F64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    long long* sk = (long long*)smem;
    long long* sa0 = sk + kPartTile;
    long long* sa1 = sa0 + kPartTile;                                   // AV only
    uint8_t* sp = (uint8_t*)(sa0 + (AV ? 2 : 1) * kPartTile);
    uint8_t* sb = sp + kPartTile;
    __shared__ uint32_t lh[kPartBuckets], ls[kPartBuckets];
    __shared__ int64_t lbase[kPartBuckets];
    const int64_t g = blockIdx.x;
    int64_t lo, hi;
    int b1 = 0;
    if constexpr (PASS == 1) {
        lo = g * kPartTile;
        hi = min(a.n, lo + (int64_t)kPartTile);
    } else {
        if (!pass2_tile(a, g, b1, lo, hi)) return;
    }
    const bool single = a.d2_bits == 0;
    int64_t* o_key = (PASS == 2 || single) ? a.e_key : a.p1_key;
    int64_t* o_a0 = (PASS == 2 || single) ? a.e_a0 : a.p1_a0;
    int64_t* o_a1 = (PASS == 2 || single) ? a.e_a1 : a.p1_a1;
    uint8_t* o_pos = (PASS == 2 || single) ? a.e_pos : a.p1_pos;
    const uint32_t* crow = (PASS == 1 ? a.p_counts1 : a.p_counts2) + g * kPartBuckets;
    const int nb = PASS == 1 ? (1 << a.d1_bits) : (1 << a.d2_bits);
    for (int b = threadIdx.x; b < kPartBuckets; b += blockDim.x) {
        lh[b] = 0;
        if (b < nb) {
            const int64_t* base = PASS == 1 ? (single ? a.rg_base : a.p1_base) : a.rg_base + ((int64_t)b1 << a.d2_bits);
            lbase[b] = base[b] + crow[b];
        }
    }
    __syncthreads();
    unsigned long long late = 0, flags = 0, occ = 0;
    const int64_t m2 = ((int64_t)1 << a.d2_bits) - 1;
    int64_t key[kPartItems], c0[kPartItems], c1[kPartItems];
    uint32_t pos[kPartItems], rank[kPartItems];
    int bk[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        const int64_t i = lo + it * kPartThreads + threadIdx.x;
        bk[it] = -1;
        key[it] = 0; c0[it] = 0; c1[it] = 0; pos[it] = 0;
        if constexpr (PASS == 1) {
            int st = REC_SKIP;
            int64_t pane = 0;
            if (i < hi) {
                key[it] = a.key[i];
                st = classify<AGG>(a, a.ts[i], a.val ? a.val[i] : 0, pos[it], pane, c0[it], c1[it], late, flags);
            }
            if (st == REC_RING) {
                if (key[it] == kEmptyKey) {  // sentinel slot: rare, straight atomics
                    cell_atomic<AGG>(pt_cell(a.t, a.t.cap, pos[it]), c0[it], c1[it]);
                    mask_set<AGG>(a.t, a.t.cap, pos[it]);
                    occ |= 1ull << pos[it];
                } else {
                    bk[it] = (int)(rgn_of(a.t, key[it]) >> a.d2_bits);
                    occ |= 1ull << pos[it];
                }
            }
            defer_write(a, st == REC_DEFER, key[it], pane, c0[it], c1[it]);
        } else {
            if (i < hi) {
                key[it] = a.p1_key[i];
                c0[it] = a.p1_a0[i];
                if constexpr (AV) c1[it] = a.p1_a1[i];
                pos[it] = a.p1_pos[i];
                bk[it] = (int)(rgn_of(a.t, key[it]) & m2);
            }
        }
        if (bk[it] >= 0) rank[it] = atomicAdd(&lh[bk[it]], 1u);
    }
    __syncthreads();
    scan_buckets(lh, ls, nb);
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {
        if (bk[it] < 0) continue;
        const uint32_t j = ls[bk[it]] + rank[it];
        sk[j] = key[it];
        sa0[j] = c0[it];
        if constexpr (AV) sa1[j] = c1[it];
        sp[j] = (uint8_t)pos[it];
        sb[j] = (uint8_t)bk[it];
    }
    __syncthreads();
    const uint32_t cnt = ls[nb - 1] + lh[nb - 1];
    for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) {
        const int b = sb[j];
        const int64_t dst = lbase[b] + (int64_t)(j - ls[b]);
        o_key[dst] = sk[j];
        o_a0[dst] = sa0[j];
        if constexpr (AV) o_a1[dst] = sa1[j];
        o_pos[dst] = sp[j];
    }
    if constexpr (PASS == 1) block_commit(a.st, late, 0, flags, occ);
}

// apply: one workgroup per region; keys / mask / up to two active pane arrays in LDS
// Copy n int64 words (n even, both ends 16-B aligned) with 16-byte accesses.
__device__ __forceinline__ void copy_words(long long* __restrict__ d, const long long* __restrict__ s, int64_t n) {
    const int64_t n2 = n >> 1;
    const long2* s2 = reinterpret_cast<const long2*>(s);
    long2* d2 = reinterpret_cast<long2*>(d);
    for (int64_t w = threadIdx.x; w < n2; w += blockDim.x) d2[w] = s2[w];
}

// Records per thread loaded in the prologue together with the region's state, so the
// two latencies overlap (a region holds ~1200 records of a 10M batch at 8192 regions).
constexpr int kApplyPre = 4;

template <int AGG>
__global__ void __launch_bounds__(512) k_rgn_apply(IngestArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool M = uses_mask<AGG>();
    constexpr bool AV = AGG == GW_AVG_I64 || AGG == GW_AVG_F64;
    const int64_t r = blockIdx.x;
    const int64_t lo = a.rg_base[r], hi = a.rg_base[r + 1];
    if (lo == hi) return;  // uniform: no records for this region in this batch
    const int64_t S = pt_S(a.t);
    const int W = a.t.words;
    long long* lkeys = (long long*)smem;
    const int64_t MW = pt_mask_words(a.t);       // 0 unless M
    uint8_t* lmask = (uint8_t*)(lkeys + S);
    long long* lcell = lkeys + S + MW;           // [2][S][W]
    // dirty 128-B lines of the key and mask arrays (S <= 2048: <= 128 key lines)
    __shared__ uint32_t s_kdirty[4], s_mdirty[4];
    // the (up to) two pane positions this batch touches
    const unsigned long long bocc = *(volatile unsigned long long*)a.batch_occ;
    const int act0 = bocc ? __ffsll((long long)bocc) - 1 : -1;
    const unsigned long long rest = bocc & (bocc - 1);
    const int act1 = rest ? __ffsll((long long)rest) - 1 : -1;
    int64_t* gkeys = pt_region(a.t, r);
    int64_t* gmask = gkeys + S;
    const int msh = a.t.mask_shift;
    // prologue: this thread's first records + the region state, all loads in flight
    int64_t pk[kApplyPre], p0[kApplyPre], p1[kApplyPre];
    uint32_t pp[kApplyPre];
#pragma unroll
    for (int q = 0; q < kApplyPre; ++q) {
        const int64_t e = lo + q * (int64_t)blockDim.x + threadIdx.x;
        pk[q] = 0; p0[q] = 0; p1[q] = 1; pp[q] = 0;
        if (e < hi) {
            pk[q] = a.e_key[e];
            p0[q] = a.e_a0[e];
            if constexpr (AV) p1[q] = a.e_a1[e];
            pp[q] = a.e_pos[e];
        }
    }
    copy_words(lkeys, (const long long*)gkeys, S);
    if constexpr (M) copy_words((long long*)lmask, (const long long*)gmask, MW);
    for (int ai = 0; ai < 2; ++ai) {
        const int p = ai ? act1 : act0;
        if (p < 0) continue;
        long long* dst = lcell + (int64_t)ai * S * W;
        if ((a.ring_fresh >> p) & 1) {  // position retired since its last use: all identity
            const int64_t id0 = identity0(AGG);
            for (int64_t w = threadIdx.x; w < S * W; w += blockDim.x) dst[w] = (W == 2 && (w & 1)) ? 0 : id0;
        } else {
            copy_words(dst, (const long long*)pt_cell(a.t, r << a.t.log2S, p), S * W);
        }
    }
    if (threadIdx.x < 4) { s_kdirty[threadIdx.x] = 0; s_mdirty[threadIdx.x] = 0; }
    __syncthreads();
    unsigned long long ins = 0, flags = 0;
    auto apply_one = [&](int64_t key, int64_t c0, int64_t c1, uint32_t pos, int64_t& pane) -> bool {
        int64_t j = pt_home(a.t, slot_hash(key));
        int64_t found = -1;
        for (int64_t p = 0; p < S; ++p) {
            const long long k = lkeys[j];
            if (k == key) { found = j; break; }
            if (k == kEmptyKey) {
                const unsigned long long prev = atomicCAS((unsigned long long*)&lkeys[j],
                                                          (unsigned long long)kEmptyKey, (unsigned long long)key);
                if (prev == (unsigned long long)kEmptyKey) {
                    found = j;
                    ins++;
                    atomicOr(&s_kdirty[j >> 9], 1u << ((j >> 4) & 31));
                    break;
                }
                if ((int64_t)prev == key) { found = j; break; }
            }
            j = (j + 1) & (S - 1);
        }
        if (found < 0) {  // region full: park the record, the host grows the table
            flags |= GW_DF_TABLE_FULL;
            const int64_t rel = ((int64_t)pos - a.b_pos + a.t.ring) % a.t.ring;
            pane = a.p_late + (int64_t)a.delta + rel;
            return true;
        }
        const int ai = (int)pos == act0 ? 0 : ((int)pos == act1 ? 1 : -1);
        if (ai >= 0) {
            long long* c = lcell + ((int64_t)ai * S + found) * W;
            lds_cell_add<AGG>(c, c + (W == 2 ? 1 : 0), c0, c1);
        } else {  // a third pane in one batch: device atomics on this region's cells
            cell_atomic<AGG>(pt_cell(a.t, (r << a.t.log2S) + found, (int)pos), c0, c1);
        }
        if constexpr (M) {
            if (mask_set_bit(lmask, found, msh, pos)) {
                const int64_t line = (found << msh) >> 7;
                atomicOr(&s_mdirty[line >> 5], 1u << (line & 31));
            }
        }
        return false;
    };
#pragma unroll
    for (int q = 0; q < kApplyPre; ++q) {
        const int64_t e = lo + q * (int64_t)blockDim.x + threadIdx.x;
        int64_t pane = 0;
        const bool defer = e < hi && apply_one(pk[q], p0[q], p1[q], pp[q], pane);
        defer_write(a, defer, pk[q], pane, p0[q], p1[q]);
    }
    for (int64_t e0 = lo + kApplyPre * (int64_t)blockDim.x; e0 < hi; e0 += blockDim.x) {
        const int64_t e = e0 + threadIdx.x;
        bool defer = false;
        int64_t key = 0, pane = 0, c0 = 0, c1 = 1;
        if (e < hi) {
            key = a.e_key[e];
            c0 = a.e_a0[e];
            if constexpr (AV) c1 = a.e_a1[e];
            defer = apply_one(key, c0, c1, a.e_pos[e], pane);
        }
        defer_write(a, defer, key, pane, c0, c1);
    }
    __syncthreads();
    // write back: dirty 128-B lines of keys / mask, every line of the active pane arrays
    {
        const long2* sk = reinterpret_cast<const long2*>(lkeys);
        long2* dk = reinterpret_cast<long2*>(gkeys);
        for (int64_t w = threadIdx.x; w < S / 2; w += blockDim.x) {
            const int64_t line = w >> 3;
            if (s_kdirty[line >> 5] & (1u << (line & 31))) dk[w] = sk[w];
        }
    }
    if constexpr (M) {
        const long2* sm = reinterpret_cast<const long2*>(lmask);
        long2* dm = reinterpret_cast<long2*>(gmask);
        for (int64_t w = threadIdx.x; w < MW / 2; w += blockDim.x) {
            const int64_t line = w >> 3;
            if (s_mdirty[line >> 5] & (1u << (line & 31))) dm[w] = sm[w];
        }
    }
    for (int ai = 0; ai < 2; ++ai) {
        const int p = ai ? act1 : act0;
        if (p < 0) continue;
        copy_words((long long*)pt_cell(a.t, r << a.t.log2S, p), lcell + (int64_t)ai * S * W, S * W);
    }
    block_commit(a.st, 0, ins, flags, 0);
}

// ---------------------------------------------------------------------------
// deferred list, fire, evict, rehash
// ---------------------------------------------------------------------------
template <int AGG>
__global__ void __launch_bounds__(256) k_merge_deferred(MergeArgs a) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t R = a.t.ring;
    unsigned long long ins = 0, flags = 0, occ = 0;
    for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < a.n; base += stride) {
        const int64_t i = base + threadIdx.x;
        bool keep = false;
        int64_t key = 0, pane = 0, c0 = 0, c1 = 0;
        if (i < a.n) {
            key = a.i_key[i];
            pane = a.i_pane[i];
            c0 = a.i_a0[i];
            c1 = a.i_a1[i];
            const bool in_ring = pane >= a.b && (uint64_t)pane - (uint64_t)a.b < (uint64_t)R;
            if (in_ring) {
                int64_t pos = a.b_pos + (pane - a.b);
                if (pos >= R) pos -= R;
                bool inserted;
                const int64_t g = pt_find_or_insert(a.t, key, inserted);
                ins += inserted;
                if (g < 0) {
                    flags |= GW_DF_TABLE_FULL;
                    keep = true;
                } else {
                    cell_atomic<AGG>(pt_cell(a.t, g, (int)pos), c0, c1);
                    mask_set<AGG>(a.t, g, (uint32_t)pos);
                    occ |= 1ull << pos;
                }
            } else {
                keep = true;
            }
        }
        const unsigned long long off = wave_reserve(&a.st->n_deferred, keep);
        if (keep) {
            a.d_key[off] = key;
            a.d_pane[off] = pane;
            a.d_a0[off] = c0;
            a.d_a1[off] = c1;
        }
    }
    block_commit(a.st, 0, ins, flags, occ);
}

__global__ void __launch_bounds__(256) k_deferred_min(const int64_t* pane, int64_t n, DevStatus* st) {
    long long m = INT64_MAX;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        m = pane[i] < m ? pane[i] : m;
    for (int o = 32; o > 0; o >>= 1) {
        long long x = __shfl_xor(m, o);
        m = x < m ? x : m;
    }
    if (__lane_id() == 0 && m != INT64_MAX) atomicMin(&st->def_min_pane, m);
}

// Fire pass: one streaming sweep over all slots emits every (key, window) with a
// non-null pane among the nwin windows of this pass, then retires the panes no later
// window covers (clearAllState).  Each block sweeps a contiguous chunk of slots; the
// SoA layout makes every key / mask / cell access coalesced.  Rows are staged in LDS
// and flushed with one device atomic per flush.  Retired pane arrays are overwritten
// with the identity unconditionally (full-line coalesced stores).
template <int AGG>
__global__ void __launch_bounds__(256) k_fire(FireArgs a) {
    __shared__ RowStage rs;
    const int64_t nslots = a.t.cap + 1;
    const int64_t id0 = identity0(AGG);
    const int W = a.t.words;
    if (threadIdx.x == 0) rs.cnt = 0;
    if (blockIdx.x == 0 && threadIdx.x < kShards) atomicAnd(&a.st->sh[threadIdx.x].occ, ~a.rmask);
    __syncthreads();
    const int64_t chunk = ((nslots + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
    const int64_t c0 = blockIdx.x * chunk, c1 = min(nslots, c0 + chunk);
    for (int64_t base = c0; base < c1; base += blockDim.x) {
        const int64_t g = base + threadIdx.x;
        int64_t key = kEmptyKey;
        uint64_t mask = 0;
        const bool live = g < c1;
        if (live) {
            key = *pt_key(a.t, g);
            mask = presence<AGG>(a.t, g);
        }
        for (int w = 0; w < a.nwin; ++w) {
            const bool flush = rs.cnt + blockDim.x > kRowStage;  // uniform: read before any append
            __syncthreads();
            if (flush) stage_flush(rs, &a.st->rows, a.o_key, a.o_start, a.o_end, a.o_res);
            uint64_t m = mask & a.wmask[w];
            if (m) {
                int64_t r0 = id0, r1 = 0;
                while (m) {
                    const int pos = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    const int64_t* c = pt_cell(a.t, g, pos);
                    fold_cell(AGG, r0, r1, c[0], W == 2 ? c[1] : 0);
                }
                const unsigned j = atomicAdd(&rs.cnt, 1u);
                const int64_t st = a.start0 + (int64_t)w * a.slide;
                rs.k[j] = key;
                rs.s[j] = st;
                rs.e[j] = st + a.size;
                rs.r[j] = cell_result(AGG, r0, r1);
            }
            __syncthreads();
        }
        if (live && a.rmask) {
            if constexpr (uses_mask<AGG>()) {
                if (mask & a.rmask) pt_mask_put(a.t, g, mask & ~a.rmask);
            }
            uint64_t m = a.rmask;
            while (m) {
                const int pos = __ffsll((long long)m) - 1;
                m &= m - 1;
                int64_t* c = pt_cell(a.t, g, pos);
                c[0] = id0;
                if (W == 2) c[1] = 0;
            }
        }
    }
    stage_flush(rs, &a.st->rows, a.o_key, a.o_start, a.o_end, a.o_res);
}

// Move the cells of ring positions `emask` to the deferred list (ring re-base down).
template <int AGG>
__global__ void __launch_bounds__(256) k_evict(EvictArgs a) {
    const int64_t nslots = a.t.cap + 1;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t id0 = identity0(AGG);
    const int W = a.t.words;
    if (blockIdx.x == 0 && threadIdx.x < kShards) atomicAnd(&a.st->sh[threadIdx.x].occ, ~a.emask);
    for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < nslots; base += stride) {
        const int64_t g = base + threadIdx.x;
        uint64_t m = 0;
        int64_t key = 0;
        if (g < nslots) {
            key = *pt_key(a.t, g);
            m = presence<AGG>(a.t, g) & a.emask;
        }
        unsigned long long off = wave_reserve_n(&a.st->n_deferred, (unsigned)__popcll(m));
        if (m) {
            if constexpr (uses_mask<AGG>()) pt_mask_put(a.t, g, pt_mask_get(a.t, g) & ~a.emask);
            while (m) {
                const int pos = __ffsll((long long)m) - 1;
                m &= m - 1;
                int64_t* c = pt_cell(a.t, g, pos);
                a.d_key[off] = key;
                a.d_pane[off] = a.pane_of_pos[pos];
                a.d_a0[off] = c[0];
                a.d_a1[off] = W == 2 ? c[1] : 0;
                off++;
                c[0] = id0;
                if (W == 2) c[1] = 0;
            }
        }
    }
}

// Re-hash live slots into a fresh (larger) table; dead keys are dropped.
__global__ void __launch_bounds__(256) k_rehash(PaneTable o, PaneTable n, DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g <= o.cap; g += (int64_t)gridDim.x * blockDim.x) {
        if (presence_rt(o, g) == 0) continue;
        const int64_t key = g == o.cap ? kEmptyKey : *pt_key(o, g);
        bool inserted;
        const int64_t h = pt_find_or_insert(n, key, inserted);
        if (h < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        ins += inserted;
        if (o.has_mask) pt_mask_put(n, h, pt_mask_get(o, g));
        for (int r = 0; r < o.ring; ++r) {
            const int64_t* s = pt_cell(o, g, r);
            int64_t* d = pt_cell(n, h, r);
            d[0] = s[0];
            if (o.words == 2) d[1] = s[1];
        }
    }
    block_commit(st, 0, ins, flags, 0);
}

__global__ void __launch_bounds__(256) k_count_live(PaneTable t, unsigned long long* out) {
    unsigned long long c = 0;
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g <= t.cap; g += (int64_t)gridDim.x * blockDim.x)
        c += presence_rt(t, g) != 0;
    c = wave_sum(c);
    if (__lane_id() == 0 && c) atomicAdd(out, c);
}

// Status word writes, ordered on the stream (no host sync).
__global__ void k_status_set(DevStatus* st, int word, unsigned long long v, int shard_field) {
    if (shard_field >= 0) {
        if (threadIdx.x < kShards) reinterpret_cast<unsigned long long*>(&st->sh[threadIdx.x])[shard_field] = v;
    } else if (threadIdx.x == 0) {
        reinterpret_cast<unsigned long long*>(st)[word] = v;
    }
}

// ---------------------------------------------------------------------------
// host-side launchers (template dispatch on the aggregate)
// ---------------------------------------------------------------------------
#define GW_AGG_SWITCH(agg, CALL)                  \
    switch (agg) {                                \
    case GW_COUNT: CALL(GW_COUNT); break;         \
    case GW_SUM_I64: CALL(GW_SUM_I64); break;     \
    case GW_SUM_F64: CALL(GW_SUM_F64); break;     \
    case GW_MIN_I64: CALL(GW_MIN_I64); break;     \
    case GW_MAX_I64: CALL(GW_MAX_I64); break;     \
    case GW_MIN_F64: CALL(GW_MIN_F64); break;     \
    case GW_MAX_F64: CALL(GW_MAX_F64); break;     \
    case GW_AVG_I64: CALL(GW_AVG_I64); break;     \
    case GW_AVG_F64: CALL(GW_AVG_F64); break;     \
    case GW_SUM_I32: CALL(GW_SUM_I32); break;     \
    default: break;                               \
    }

static inline int grid_for(int64_t n, int per_thread = 1) {
    int64_t g = ((n + per_thread - 1) / per_thread + 255) / 256;
    if (g < 1) g = 1;
    if (g > 256 * 8) g = 256 * 8;  // 8 blocks (32 waves) per CU, grid-stride the rest
    return (int)g;
}

int64_t region_scratch_tiles(int64_t n) { return std::max<int64_t>(1, (n + kPartTile - 1) / kPartTile); }

hipError_t launch_table_init(const PaneTable& t, hipStream_t s) {
#define L(A) hipLaunchKernelGGL(k_table_init<A>, dim3(grid_for(t.cap + 1)), dim3(256), 0, s, t)
    GW_AGG_SWITCH(t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_ingest(const IngestArgs& a, int path, int unroll, hipStream_t s) {
    if (path == 1) {
        const int g = grid_for(a.n, kPreaggItems);
#define L(A) hipLaunchKernelGGL(k_ingest_preagg<A>, dim3(g), dim3(256), 0, s, a)
        GW_AGG_SWITCH(a.t.agg, L);
#undef L
    } else if (path == 2) {
        const int64_t tiles1 = region_scratch_tiles(a.n);
        const int64_t tiles2 = tiles1 + kPartBuckets;
        const bool single = a.d2_bits == 0;
        const int nb1 = 1 << a.d1_bits;
        const size_t part_lds = (size_t)kPartTile * 8 * (a.t.words == 2 ? 3 : 2) + 2 * kPartTile;
        const int64_t S = pt_S(a.t);
        const size_t apply_lds = (size_t)(S + pt_mask_words(a.t)) * 8 + (size_t)2 * S * a.t.words * 8;
        int64_t* b1 = single ? a.rg_base : a.p1_base;
        // beyond the 64 KB default: opt in (gfx950 has 160 KB of LDS per CU)
#define L(A)                                                                                                    \
    hipFuncSetAttribute((const void*)k_part_scatter<A, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,          \
                        (int)part_lds);                                                                         \
    hipFuncSetAttribute((const void*)k_part_scatter<A, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,          \
                        (int)part_lds);                                                                         \
    hipFuncSetAttribute((const void*)k_rgn_apply<A>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)apply_lds); \
    hipLaunchKernelGGL((k_part_hist<A, 1>), dim3((unsigned)tiles1), dim3(kPartThreads), 0, s, a);             \
    hipLaunchKernelGGL(k_part_cols1, dim3(nb1), dim3(256), 0, s, a.p_counts1, tiles1, b1);                     \
    hipLaunchKernelGGL(k_rgn_bases, dim3(1), dim3(1024), 0, s, b1, (int64_t)nb1, single ? nullptr : a.p2_tile0); \
    hipLaunchKernelGGL((k_part_scatter<A, 1>), dim3((unsigned)tiles1), dim3(kPartThreads), part_lds, s, a);   \
    if (!single) {                                                                                              \
        hipLaunchKernelGGL((k_part_hist<A, 2>), dim3((unsigned)tiles2), dim3(kPartThreads), 0, s, a);         \
        hipLaunchKernelGGL(k_part_cols2, dim3((unsigned)((a.t.nreg + 255) / 256)), dim3(256), 0, s, a);       \
        hipLaunchKernelGGL(k_rgn_bases, dim3(1), dim3(1024), 0, s, a.rg_base, a.t.nreg, (int64_t*)nullptr);   \
        hipLaunchKernelGGL((k_part_scatter<A, 2>), dim3((unsigned)tiles2), dim3(kPartThreads), part_lds, s, a); \
    }                                                                                                           \
    hipLaunchKernelGGL(k_rgn_apply<A>, dim3((unsigned)a.t.nreg), dim3(512), apply_lds, s, a)
        GW_AGG_SWITCH(a.t.agg, L);
#undef L
    } else if (unroll == 4) {
        const int g = grid_for(a.n, 4);
#define L(A) hipLaunchKernelGGL((k_ingest<A, 4>), dim3(g), dim3(256), 0, s, a)
        GW_AGG_SWITCH(a.t.agg, L);
#undef L
    } else if (unroll == 2) {
        const int g = grid_for(a.n, 2);
#define L(A) hipLaunchKernelGGL((k_ingest<A, 2>), dim3(g), dim3(256), 0, s, a)
        GW_AGG_SWITCH(a.t.agg, L);
#undef L
    } else {
        const int g = grid_for(a.n, 1);
#define L(A) hipLaunchKernelGGL((k_ingest<A, 1>), dim3(g), dim3(256), 0, s, a)
        GW_AGG_SWITCH(a.t.agg, L);
#undef L
    }
    return hipGetLastError();
}

hipError_t launch_merge_deferred(const MergeArgs& a, hipStream_t s) {
#define L(A) hipLaunchKernelGGL(k_merge_deferred<A>, dim3(grid_for(a.n)), dim3(256), 0, s, a)
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_deferred_min(const int64_t* pane, int64_t n, DevStatus* st, hipStream_t s) {
    hipLaunchKernelGGL(k_deferred_min, dim3(grid_for(n)), dim3(256), 0, s, pane, n, st);
    return hipGetLastError();
}

hipError_t launch_fire(const FireArgs& a, hipStream_t s) {
    const int fg = (int)std::min<int64_t>(1024, std::max<int64_t>(1, (a.t.cap + 1 + 255) / 256));
#define L(A) hipLaunchKernelGGL(k_fire<A>, dim3(fg), dim3(256), 0, s, a)
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_evict(const EvictArgs& a, hipStream_t s) {
#define L(A) hipLaunchKernelGGL(k_evict<A>, dim3(grid_for(a.t.cap + 1)), dim3(256), 0, s, a)
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_status_set(DevStatus* st, int word, unsigned long long v, int shard_field, hipStream_t s) {
    hipLaunchKernelGGL(k_status_set, dim3(1), dim3(64), 0, s, st, word, v, shard_field);
    return hipGetLastError();
}

hipError_t launch_count_live(const PaneTable& t, unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(k_count_live, dim3(grid_for(t.cap + 1)), dim3(256), 0, s, t, out);
    return hipGetLastError();
}

hipError_t launch_rehash(const PaneTable& o, const PaneTable& n, DevStatus* st, hipStream_t s) {
    hipLaunchKernelGGL(k_rehash, dim3(grid_for(o.cap + 1)), dim3(256), 0, s, o, n, st);
    return hipGetLastError();
}

}  // namespace gw
