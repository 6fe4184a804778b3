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
#include <hip/hip_ext.h>
#include <type_traits>
#include "gw_kernels.h"

#include <algorithm>
#include <mutex>
#include <vector>

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

__device__ __forceinline__ int64_t floor_div_d(int64_t a, int64_t b) {
    const int64_t q = a / b;
    return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}

// Per-record classification: late / parked (outside the pane ring) / in ring / re-fire
// (allowed lateness > 0: the pane belongs to a fired window that is not cleaned yet).
enum { REC_SKIP = 0, REC_RING = 1, REC_DEFER = 2, REC_REFIRE = 3, REC_LATE = 4 };
template <int AGG, bool GAP = true>
__device__ __forceinline__ int classify(const IngestArgs& a, int64_t ts, int64_t v, uint32_t& pos, int64_t& pane,
                                        int64_t& c0, int64_t& c1, unsigned long long& late,
                                        unsigned long long& flags) {
    if (ts == INT64_MIN) { flags |= GW_DF_NO_TS; return REC_SKIP; }
    if (ts < a.t_late) {  // every window of the record is late: isSkippedElement && isElementLate
        if (!a.late_exact) { flags |= GW_DF_RANGE; return REC_SKIP; }
        if (GAP && a.gap_size) {  // t_late is a pane boundary: the record's offset into its pane
            const uint64_t r = ((uint64_t)a.t_late - (uint64_t)ts) % (uint64_t)a.gap_w;
            const uint64_t off = r ? (uint64_t)a.gap_w - r : 0;
            // no window: isSkippedElement, and late only by its own timestamp
            if (off >= (uint64_t)a.gap_size && ts > a.gap_late) return REC_SKIP;
        }
        if (a.cls_J > 1) {  // window class: only the class of the record's last window reports it
            // (wrapping subtraction: timestamps within |offset| of Long.MIN_VALUE wrap as in Java)
            const int64_t k = floor_div_d((int64_t)((uint64_t)ts - (uint64_t)a.cls_off), a.cls_slide);
            int64_t c = k % a.cls_J;
            if (c < 0) c += a.cls_J;
            if (c != a.cls_j) return REC_SKIP;
        }
        if (a.lo_key) return REC_LATE;  // sideOutputLateData: the record goes to the side output
        late++;                         // numLateRecordsDropped (WindowOperator.java:440-446)
        return REC_SKIP;
    }
    const uint64_t R = (uint64_t)a.t.ring;
    const uint64_t q = udiv64((uint64_t)ts - (uint64_t)a.t_late, a.div);
    // between two windows (size < slide): assignWindows gives the record no window and it is
    // not late, so processElement does nothing with it
    if (GAP && a.gap_size && (uint64_t)ts - (uint64_t)a.t_late - q * (uint64_t)a.gap_w >= (uint64_t)a.gap_size)
        return REC_SKIP;
    record_cell(AGG, v, c0, c1);
    pane = a.p_late + (int64_t)q;
    if (q < a.q_refire) return REC_REFIRE;
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

// Late record with a late-data side output: the record itself, as processElement passes it
// to sideOutput (WindowOperator.java:440-446, 587-588).
__device__ __forceinline__ void late_write(const IngestArgs& a, bool lo, int64_t key, int64_t i) {
    const unsigned long long off = wave_reserve(&a.st->n_late_out, lo);
    if (lo) {
        a.lo_key[off] = key;
        a.lo_ts[off] = a.ts[i];
        a.lo_val[off] = a.val ? a.val[i] : 0;
    }
}

// Late record of a fired, not yet cleaned window: onto the re-fire list with its
// arrival number (processed in order at the next watermark, k_refire).
__device__ __forceinline__ void refire_write(const IngestArgs& a, bool rf, int64_t key, int64_t pane, int64_t c0,
                                             int64_t c1, int64_t i) {
    const unsigned long long off = wave_reserve(&a.st->n_refire, rf);
    if (rf) {
        a.rf_key[off] = key;
        a.rf_pane[off] = pane;
        a.rf_a0[off] = c0;
        a.rf_a1[off] = c1;
        a.rf_seq[off] = a.seq0 + i;
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
        if (p) k = *kp;
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
                        ? *(pt_region(a.t, reg[u]) + home[u])
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
        for (int u = 0; u < U; ++u) {
            defer_write(a, state[u] == REC_DEFER, key[u], pane[u], c0[u], c1[u]);
            refire_write(a, state[u] == REC_REFIRE, key[u], pane[u], c0[u], c1[u],
                         base + (int64_t)u * blockDim.x + threadIdx.x);
            if (a.lo_key) late_write(a, state[u] == REC_LATE, key[u], base + (int64_t)u * blockDim.x + threadIdx.x);
        }
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

// Few live keys per batch (YSB's 100 campaigns): a persistent grid (two workgroups per CU)
// keeps, per workgroup, an LDS cache key -> table slot (kPreKeys entries: the table is probed
// once per key per workgroup, not once per record) and an LDS hash of (cached key, ring
// position) accumulators (kLdsCells), and adds them into the table once, when the workgroup's
// last tile is done.  Per 2048-record tile: every record loads up front (8 per thread); keys are
// claimed in the cache (phase A), the new keys are probed in the table by one thread each
// (phase B), then records fold into the LDS cells (phase C).  A key the cache cannot hold, or a
// cell the LDS hash cannot hold, goes straight to the table with one device atomic.  So the
// table sees ~(workgroups x live cells) atomics per batch instead of one per record or per
// tile (round 4: one flush per 2048-record tile put ~3.3K atomics on each hot cell).
constexpr int kPreKeys = 1024;

// Experiment builds only (flink_amd.build --define GW_PREAGG_EXP=n --out ...), results
// discarded: 1 no key cache, 2 no LDS cells, 4 no table adds.  The product library is built with 0.
#ifndef GW_PREAGG_EXP
#define GW_PREAGG_EXP 0
#endif
template <int AGG>
__global__ void __launch_bounds__(256) k_ingest_preagg(IngestArgs a) {
    constexpr int exp = GW_PREAGG_EXP;
    constexpr bool AV = AGG == GW_AVG_I64 || AGG == GW_AVG_F64;
    __shared__ long long s_key[kPreKeys];
    __shared__ long long s_g[kPreKeys + 1];  // + the sentinel key's slot (t.cap)
    __shared__ uint32_t s_cell[kLdsCells];
    __shared__ long long s_a0[kLdsCells];
    __shared__ long long s_a1[AV ? kLdsCells : 1];
    __shared__ uint32_t s_new[kPreKeys];
    __shared__ uint32_t s_nnew[2];  // per tile parity: reset a tile ahead (no extra barrier)
    const int64_t tile = (int64_t)blockDim.x * kPreaggItems;
    const uint32_t R = (uint32_t)a.t.ring;
    const int64_t id0 = identity0(AGG);
    unsigned long long late = 0, ins = 0, flags = 0, occ = 0, cells = 0;
    for (int j = threadIdx.x; j < kLdsCells; j += blockDim.x) {
        s_cell[j] = ~0u;
        s_a0[j] = id0;
        if constexpr (AV) s_a1[j] = 0;
    }
    for (int j = threadIdx.x; j < kPreKeys; j += blockDim.x) s_key[j] = kEmptyKey;
    if (threadIdx.x == 0) {
        s_g[kPreKeys] = a.t.cap;
        s_nnew[0] = s_nnew[1] = 0;
    }
    __syncthreads();
    int par = 0;
    // the next tile's inputs load while this tile is processed (two workgroups per CU do not
    // hide a tile's load latency on their own)
    int64_t nk[kPreaggItems], nt[kPreaggItems], nv[kPreaggItems];
    auto load_tile = [&](int64_t t0) {
#pragma unroll
        for (int it = 0; it < kPreaggItems; ++it) {
            const int64_t i = t0 + (int64_t)it * blockDim.x + threadIdx.x;
            const bool ok = i < a.n;
            nk[it] = ok ? a.key[i] : 0;
            nt[it] = ok ? a.ts[i] : 0;
            nv[it] = ok && a.val ? a.val[i] : 0;
        }
    };
    load_tile(blockIdx.x * tile);
    for (int64_t t0 = blockIdx.x * tile; t0 < a.n; t0 += (int64_t)gridDim.x * tile, par ^= 1) {
        int64_t key[kPreaggItems], pane[kPreaggItems], c0[kPreaggItems], c1[kPreaggItems];
        int64_t tsv[kPreaggItems], vv[kPreaggItems];
        uint32_t pos[kPreaggItems];
        int state[kPreaggItems], lk[kPreaggItems];
#pragma unroll
        for (int it = 0; it < kPreaggItems; ++it) {
            key[it] = nk[it];
            tsv[it] = nt[it];
            vv[it] = nv[it];
        }
        if (t0 + (int64_t)gridDim.x * tile < a.n) load_tile(t0 + (int64_t)gridDim.x * tile);
#pragma unroll
        for (int it = 0; it < kPreaggItems; ++it) {
            const int64_t i = t0 + (int64_t)it * blockDim.x + threadIdx.x;
            state[it] = REC_SKIP;
            pane[it] = 0; c0[it] = 0; c1[it] = 0; pos[it] = 0;
            if (i < a.n) state[it] = classify<AGG>(a, tsv[it], vv[it], pos[it], pane[it], c0[it], c1[it], late, flags);
        }
        // phase A: each record's key in the cache (claimed by CAS on first sight)
#pragma unroll
        for (int it = 0; it < kPreaggItems; ++it) {
            lk[it] = -1;
            if (state[it] != REC_RING) continue;
            if (key[it] == kEmptyKey || (exp & 1)) { lk[it] = kPreKeys; continue; }
            uint32_t h = (uint32_t)slot_hash(key[it]) & (kPreKeys - 1);
            for (int p = 0; p < 16; ++p) {
                long long cur = s_key[h];
                if (cur == kEmptyKey) {
                    cur = (long long)atomicCAS((unsigned long long*)&s_key[h], (unsigned long long)kEmptyKey,
                                               (unsigned long long)key[it]);
                    if (cur == kEmptyKey) s_new[atomicAdd(&s_nnew[par], 1u)] = h;
                }
                if (cur == kEmptyKey || cur == key[it]) { lk[it] = (int)h; break; }
                h = (h + 1) & (kPreKeys - 1);
            }
        }
        __syncthreads();
        // phase B: the keys new to the cache find their table slots
        const uint32_t nn = s_nnew[par];
        if (threadIdx.x == 0) s_nnew[par ^ 1] = 0;  // last read in the previous tile's phase B
        for (uint32_t q = threadIdx.x; q < nn; q += blockDim.x) {
            const uint32_t h = s_new[q];
            bool inserted;
            const int64_t g = pt_find_or_insert(a.t, s_key[h], inserted);
            ins += inserted;
            if (g < 0) flags |= GW_DF_TABLE_FULL;
            s_g[h] = g;
        }
        __syncthreads();
        // phase C: fold into the LDS cells
#pragma unroll
        for (int it = 0; it < kPreaggItems; ++it) {
            const int64_t i = t0 + (int64_t)it * blockDim.x + threadIdx.x;
            if (state[it] == REC_RING) {
                int64_t g;
                if (lk[it] >= 0) {
                    g = s_g[lk[it]];
                } else {  // not cached: the table directly
                    bool inserted;
                    g = pt_find_or_insert(a.t, key[it], inserted);
                    ins += inserted;
                }
                if (g < 0) {
                    flags |= GW_DF_TABLE_FULL;
                    state[it] = REC_DEFER;
                } else {
                    occ |= 1ull << pos[it];
                    bool done = false;
                    if (exp & 2) {
                        done = true;
                    } else if (lk[it] >= 0) {
                        const uint32_t cell = (uint32_t)lk[it] * R + pos[it];
                        uint32_t h = (cell * 0x9E3779B1u) >> (32 - 11);  // kLdsCells = 2^11
                        for (int p = 0; p < 32 && !done; ++p) {
                            uint32_t cur = s_cell[h];
                            if (cur == ~0u) cur = atomicCAS(&s_cell[h], ~0u, cell);
                            if (cur == ~0u || cur == cell) {
                                lds_cell_add<AGG>(&s_a0[h], &s_a1[AV ? h : 0], c0[it], c1[it]);
                                done = true;
                            }
                            h = (h + 1) & (kLdsCells - 1);
                        }
                    }
                    if (!done) {  // LDS cells saturated, or the key not cached: straight to HBM
                        cell_atomic<AGG>(pt_cell(a.t, g, pos[it]), c0[it], c1[it]);
                        mask_set<AGG>(a.t, g, pos[it]);
                    }
                }
            }
            defer_write(a, state[it] == REC_DEFER, key[it], pane[it], c0[it], c1[it]);
            refire_write(a, state[it] == REC_REFIRE, key[it], pane[it], c0[it], c1[it], i);
            if (a.lo_key) late_write(a, state[it] == REC_LATE, key[it], i);
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < kLdsCells; j += blockDim.x) {  // the workgroup's cells -> table
        const uint32_t cell = s_cell[j];
        if (cell == ~0u || (exp & 4)) continue;
        const uint32_t l = cell / R, pos = cell - l * R;
        const int64_t g = s_g[l];
        if (g < 0) continue;  // (records of an unplaced key deferred above; no cell was made)
        cells++;
        int64_t b1 = 0;
        if constexpr (AV) b1 = s_a1[j];
        cell_atomic<AGG>(pt_cell(a.t, g, pos), s_a0[j], b1);
        mask_set<AGG>(a.t, g, pos);
    }
    block_commit(a.st, late, ins, flags, occ, cells);
}

// ---------------------------------------------------------------------------
// region path: tile-local two-level bucketing, then one workgroup per region
// ---------------------------------------------------------------------------
// In-ring records are bucketed by table region (gw_kernels.h pt_key_region: bucket = the top
// rb1 bits of the key hash, region within the bucket = the next bits scaled to nsub) without
// histogram passes:
//   P1  (per watermark batch) one block per 4096-record tile classifies its records,
//       sorts them in LDS by pass-1 bucket (top d1 = rb1 hash bits) and writes the tile
//       back contiguously, plus one descriptor row: per bucket (start << 16 | count).
//   P2  (per flush, two-pass tables) block (b1, j) gathers bucket b1's runs from a group
//       of G P1 tiles, sorts them by region within the bucket (pt_sub) in LDS and writes
//       rounds of <= 4096 records, each with a descriptor row of its own.  Two small
//       plan kernels place the blocks' outputs (bucket-major) and their rounds.
//   apply  one workgroup per region gathers its runs (from the P2 rounds of its bucket,
//       or straight from the P1 tiles of a single-pass table) and applies them to an
//       LDS copy of the region's keys / mask / active pane arrays.
// Every HBM access is a contiguous run: whole tiles, runs of ~32-64 records, and the
// region state.  P1 segments of several watermark batches accumulate in the buffer and
// P2 + apply run once per fire (gw_runtime.cpp flush_buffer).
#ifndef GW_PART_THREADS
#define GW_PART_THREADS 512
#endif
constexpr int kPartThreads = GW_PART_THREADS;
constexpr int kPartItems = kPartTile / kPartThreads;

__device__ __forceinline__ int64_t rgn_of(const PaneTable& t, int64_t key) { return pt_key_region(t, slot_hash(key)); }
__device__ __forceinline__ uint32_t desc_pack(uint32_t start, uint32_t cnt) { return (start << 16) | cnt; }

// Compact records (integer aggregates; the host enables them when R <= 2^(d1-1)): 12 B per
// record instead of 17 (8 for COUNT).  The 64-bit word is the key's hash with its top d1
// bits -- the pass-1 bucket, known from where the record sits -- replaced by the ring
// position, bit 63 marking a spill; the value is 32 bits (wider values go to the deferred
// list in P1).  The hash is a bijection (slot_unhash), so the apply recovers the key.
template <int AGG>
__device__ __forceinline__ constexpr bool cmp_agg() {
    return AGG == GW_COUNT || AGG == GW_SUM_I64 || AGG == GW_SUM_I32 || AGG == GW_MIN_I64 || AGG == GW_MAX_I64 ||
           AGG == GW_AVG_I64;
}
__device__ __forceinline__ uint64_t cmp_pack(uint64_t h, uint32_t pos, int d1) {
    const int sh = 64 - d1;
    return (h & ((1ull << sh) - 1ull)) | ((uint64_t)pos << sh);
}
__device__ __forceinline__ uint64_t cmp_hash(uint64_t w, uint64_t bucket, int d1) {
    const int sh = 64 - d1;
    return (bucket << sh) | (w & ((1ull << sh) - 1ull));
}
__device__ __forceinline__ uint32_t cmp_pos(uint64_t w, int d1) { return (uint32_t)((w << 1) >> (65 - d1)); }
constexpr uint64_t kCmpSpill = 1ull << 63;

// Record formats of the region buffer (IngestArgs::fmt, fixed per flush window by the host):
// wide (key, acc word(s), ring position byte), compact (hash word + 32-bit value, above) and
// narrow -- integer aggregates whose keys fit 32 bits (28 for COUNT) and values 28 bits
// signed, ring positions < 8: the key itself, no hash, in 8 B (4 B for COUNT):
//   8 B:  lo32 = key, hi32 = value << 4 | spill << 3 | ring position
//   4 B:  key << 4 | spill << 3 | ring position                      (COUNT)
// P2 and the apply recompute the key's hash (region bits, home slot) from it.  A record that
// does not fit goes to the deferred list (exact); past 1/64 of a window's records the
// handle drops to compact records at its next window.
constexpr int kFmtWide = 0, kFmtCmp = 1, kFmtNar = 2;
constexpr int64_t kNarKeyLimit = (1ll << 32) - 2, kNarCountKeyLimit = 1ll << 28, kNarValLimit = 1ll << 27;
__device__ __forceinline__ uint64_t nar_pack(int64_t key, int64_t v, uint32_t pos) {
    return (uint64_t)(uint32_t)key | ((uint64_t)(((uint32_t)(int32_t)v << 4) | pos) << 32);
}
__device__ __forceinline__ uint32_t nar_pack32(int64_t key, uint32_t pos) { return ((uint32_t)key << 4) | pos; }
__device__ __forceinline__ int64_t nar_key(uint64_t r) { return (int64_t)(uint32_t)r; }
__device__ __forceinline__ int64_t nar_key32(uint32_t r) { return (int64_t)(r >> 4); }
__device__ __forceinline__ uint32_t nar_pos(uint32_t low_bits) { return low_bits & 7u; }
__device__ __forceinline__ bool nar_spilled(uint32_t low_bits) { return (low_bits >> 3) & 1u; }
__device__ __forceinline__ int64_t nar_val(uint64_t r) { return (int64_t)((int32_t)(uint32_t)(r >> 32) >> 4); }
constexpr uint32_t kNarSpill = 8u;  // in the low bits of hi32 (8 B) or of the record (4 B)

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

// Exclusive block scan of cnt[0..n) (n <= 2 * blockDim.x, blockDim.x = 512) into pre[],
// pre[n] = total.  Every thread calls it; ends with a barrier.
__device__ __forceinline__ void block_scan2(const uint32_t* cnt, uint32_t* pre, int n, uint32_t* wsum) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t a = 2 * t < n ? cnt[2 * t] : 0u, b = 2 * t + 1 < n ? cnt[2 * t + 1] : 0u;
    uint32_t incl = a + b;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t up = __shfl_up(incl, o);
        if (lane >= o) incl += up;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t off = 0;
    for (int q = 0; q < w; ++q) off += wsum[q];
    const uint32_t ex = off + incl - (a + b);
    if (2 * t < n) pre[2 * t] = ex;
    if (2 * t + 1 < n) pre[2 * t + 1] = ex + a;
    if (t == blockDim.x - 1) pre[n] = off + incl;
    __syncthreads();
}

// Index i of the run holding record e: pre[i] <= e < pre[i + 1] (pre ascending, n runs,
// pre[n] = total).  Runs of one bucket over a tile group are of similar length, so a guess
// proportional to e is usually right or one off: a short walk from it instead of a
// dependent binary search (7 LDS round trips at 112 runs).
// (The guess in single precision from the block's runs per record: the walk corrects any
// rounding, and a 64-bit integer division per record was ~100 VALU instructions.)
__device__ __forceinline__ int run_near(const uint32_t* pre, int n, uint32_t e, float runs_per_record) {
    int i = min(n - 1, (int)((float)e * runs_per_record));
    while (i > 0 && pre[i] > e) --i;
    while (i + 1 < n && pre[i + 1] <= e) ++i;
    return i;
}
__device__ __forceinline__ int run_of(const uint32_t* pre, int n, uint32_t e) {
    int l = 0, h = n - 1;
    while (l < h) {
        const int mid = (l + h + 1) >> 1;
        if (pre[mid] <= e) l = mid;
        else h = mid - 1;
    }
    return l;
}

// LDS image of one sorted tile: keys, accumulator words, ring positions, buckets.
struct TileLds {
    long long* k;
    long long* a0;
    long long* a1;
    uint8_t* pos;
    uint8_t* bk;
};
template <bool AV>
__device__ __forceinline__ TileLds tile_lds(unsigned char* smem) {
    TileLds s;
    s.k = (long long*)smem;
    s.a0 = s.k + kPartTile;
    s.a1 = s.a0 + kPartTile;  // AV only
    s.pos = (uint8_t*)(s.a0 + (AV ? 2 : 1) * kPartTile);
    s.bk = s.pos + kPartTile;
    return s;
}

// After a buffered P1 (same stream, one workgroup): copy the status block into the
// host's pinned slot and stamp it with the launch's sequence number.  This replaces an
// event + asynchronous copy on a side stream after every batch.  The slot stores are
// system-scope and acknowledged (vmcnt) by every wave before the barrier that precedes
// the stamp store, so no L2 write-back fence is needed.  (A last-arriver publish inside
// P1 cost ~10 us per batch: a returning atomic per workgroup on the critical path.)
__global__ void __launch_bounds__(256) k_publish_status(const DevStatus* st, DevStatus* host, unsigned long long seq) {
    constexpr int kWords = (int)(sizeof(DevStatus) / 8);
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(st);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(host);
    for (int i = threadIdx.x; i < kWords; i += blockDim.x)
        if (i != kPubSeqWord + (int)(offsetof(DevStatus, pad) / 8))
            __hip_atomic_store(&dst[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(&host->pad[kPubSeqWord], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The same from one wave at the start of a buffered P1 (workgroup 0, wave 0): the status
// as the previous launches left it -- stream order has completed them -- plus whatever
// this launch's other workgroups have already added (every field only grows or gains bits,
// so an early copy is a superset the host may absorb; gw_runtime.cpp lazy_status counts the
// launch's records as unaccounted).  Replaces a k_publish_status launch after every P1: no
// launch, no gap, no extra kernel boundary per batch.
__device__ __forceinline__ void publish_status_wave(const DevStatus* st, DevStatus* host, unsigned long long seq) {
    constexpr int kWords = (int)(sizeof(DevStatus) / 8);
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(st);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(host);
    const int lane = threadIdx.x & 63;
    for (int i = lane; i < kWords; i += 64)
        if (i != kPubSeqWord + (int)(offsetof(DevStatus, pad) / 8))
            __hip_atomic_store(&dst[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // one wave: every lane's stores acknowledged
    if (lane == 0) __hip_atomic_store(&host->pad[kPubSeqWord], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// P1: one 4096-record tile of the batch -> buffer tile a.tile0 + blockIdx.x.
// GW_P1_WAVES / GW_APPLY_WAVES: minimum waves per SIMD the register allocation must allow
// (6 = 3 workgroups of 512 per CU, as many as the LDS allows, at <= 80 VGPRs)
#ifdef GW_P1_WAVES
#define GW_P1_ATTR __attribute__((amdgpu_waves_per_eu(GW_P1_WAVES)))
#else
#define GW_P1_ATTR
#endif
#ifdef GW_APPLY_WAVES
#define GW_APPLY_ATTR __attribute__((amdgpu_waves_per_eu(GW_APPLY_WAVES)))
#else
#define GW_APPLY_ATTR
#endif
// Record i of a batch (key, timestamp, value): from the columns, or decoded from its packed
// exchange word (gw_ingest_packed_device: records [pk_from, n)).
__device__ __forceinline__ void load_record(const IngestArgs& a, int64_t i, int64_t& k, int64_t& t, int64_t& v) {
    if (a.pk_w && i >= a.pk_from) {
        unpack_word(a.pk_g, a.pk_w[i - a.pk_from], k, t, v);
        if (!a.val) v = 0;
    } else {
        k = a.key[i];
        t = a.ts[i];
        v = a.val ? a.val[i] : 0;
    }
}

// P1 body for one tile: the records' inputs are in registers (item it of thread x is record
// lo + it * THR + x); lh[] zeroed and s_occ cleared by the caller, with a barrier after.
// Classifies, ranks by pass-1 bucket (LDS atomics), sorts the tile in LDS (s) and writes it
// back with its descriptor row.
template <int AGG, int FMT, bool GAP, int THR, int IT>
__device__ __forceinline__ void p1_tile(const IngestArgs& a, int64_t g, int64_t lo, int64_t hi, int64_t (&key)[IT],
                                        const int64_t (&ts)[IT], const int64_t (&val)[IT], const TileLds& s,
                                        uint32_t* lh, uint32_t* ls, unsigned long long* s_occ,
                                        unsigned long long& late, unsigned long long& flags,
                                        unsigned long long& occ_all) {
    constexpr bool C = FMT == kFmtCmp && cmp_agg<AGG>();
    constexpr bool NR = FMT == kFmtNar && cmp_agg<AGG>();
    constexpr bool N4 = NR && AGG == GW_COUNT;  // 4-byte narrow records
    constexpr bool AV = !C && !NR && (AGG == GW_AVG_I64 || AGG == GW_AVG_F64);
    constexpr bool ACC = !(C && AGG == GW_COUNT);  // COUNT records carry no value
    int32_t* s_v32 = reinterpret_cast<int32_t*>(s.a0);  // C: 32-bit values
    uint32_t* s_r32 = reinterpret_cast<uint32_t*>(s.k);  // N4: the records
    const int nb = 1 << a.d1_bits;
    unsigned long long occ = 0, wide = 0;
    bool special = false;
    // Registers per record after classification: the key (compact: the hash word), the
    // value (32 bits for compact records), and bucket << 16 | rank in one word (~0: none).
    using V0 = std::conditional_t<C, int32_t, int64_t>;
    V0 c0[IT];
    int64_t c1[IT];
    uint32_t pos[IT], br[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int64_t i = lo + it * THR + threadIdx.x;
        int bk = -1;
        int64_t v0 = 0, v1 = 0;
        uint32_t ps = 0;
        int st = REC_SKIP;
        int64_t pane = 0;
        if (i < hi) st = classify<AGG, GAP>(a, ts[it], val[it], ps, pane, v0, v1, late, flags);
        if (C && ACC && st == REC_RING && (v0 < INT32_MIN || v0 > INT32_MAX)) {
            st = REC_DEFER;  // beyond the compact record's 32-bit value: exact via the deferred list
            wide++;
        }
        if (NR && st == REC_RING &&
            ((uint64_t)key[it] >= (uint64_t)(N4 ? kNarCountKeyLimit : kNarKeyLimit) ||
             (!N4 && (v0 < -kNarValLimit || v0 >= kNarValLimit)))) {
            st = REC_DEFER;  // beyond the narrow record: exact via the deferred list
            wide++;
        }
        if (st == REC_RING) {
            occ |= 1ull << ps;
            if (key[it] == kEmptyKey) {
                special = true;  // the sentinel slot: below
            } else {
                const uint64_t h = slot_hash(key[it]);
                bk = (int)pt_bucket(a.t, h);
                if constexpr (C) key[it] = (int64_t)cmp_pack(h, ps, a.d1_bits);  // key -> word
                if constexpr (NR) key[it] = N4 ? (int64_t)nar_pack32(key[it], ps) : (int64_t)nar_pack(key[it], v0, ps);
            }
        } else if (st != REC_SKIP) {
            special = true;  // deferred, re-fire or side-output record: below
        }
        c0[it] = (V0)v0;
        c1[it] = v1;
        pos[it] = ps;
        br[it] = bk >= 0 ? ((uint32_t)bk << 16) | atomicAdd(&lh[bk], 1u) : ~0u;
    }
    // Rare records (deferred, re-fire, side output, the sentinel key) in a second pass that
    // only waves holding one run: it re-reads and re-classifies its items (classify is
    // deterministic; its late / flag counts were taken above) and writes them out, so the
    // unrolled pass above stays small.
    if (__any(special)) {
#pragma unroll 1
        for (int it = 0; it < IT; ++it) {
            const int64_t i = lo + it * THR + threadIdx.x;
            int64_t k = 0, v0 = 0, v1 = 0, pane = 0;
            uint32_t ps = 0;
            int st = REC_SKIP;
            if (i < hi) {
                unsigned long long dl = 0, df = 0;
                int64_t t, v;
                load_record(a, i, k, t, v);
                st = classify<AGG, GAP>(a, t, v, ps, pane, v0, v1, dl, df);
                if (C && ACC && st == REC_RING && (v0 < INT32_MIN || v0 > INT32_MAX)) st = REC_DEFER;
                if (NR && st == REC_RING &&
                    ((uint64_t)k >= (uint64_t)(N4 ? kNarCountKeyLimit : kNarKeyLimit) ||
                     (!N4 && (v0 < -kNarValLimit || v0 >= kNarValLimit))))
                    st = REC_DEFER;
                if (st == REC_RING && k == kEmptyKey) {  // sentinel slot: straight atomics
                    cell_atomic<AGG>(pt_cell(a.t, a.t.cap, ps), v0, v1);
                    mask_set<AGG>(a.t, a.t.cap, ps);
                }
            }
            defer_write(a, st == REC_DEFER, k, pane, v0, v1);
            refire_write(a, st == REC_REFIRE, k, pane, v0, v1, i);
            if (a.lo_key) late_write(a, st == REC_LATE, k, i);
        }
    }
    occ_all |= occ;
    occ = wave_ior(occ);
    if (__lane_id() == 0 && occ) atomicOr(s_occ, occ);
    __syncthreads();
    scan_buckets(lh, ls, nb);
    if (threadIdx.x == 0 && *s_occ) atomicOr(a.batch_occ, *s_occ);
    __syncthreads();
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        if (br[it] == ~0u) continue;
        const uint32_t j = ls[br[it] >> 16] + (br[it] & 0xffffu);
        if constexpr (N4) {
            s_r32[j] = (uint32_t)key[it];
            continue;
        }
        s.k[j] = key[it];
        if constexpr (NR) continue;
        if constexpr (C) {
            if constexpr (ACC) s_v32[j] = c0[it];
        } else {
            s.a0[j] = c0[it];
            if constexpr (AV) s.a1[j] = c1[it];
            s.pos[j] = (uint8_t)pos[it];
        }
    }
    __syncthreads();
    const uint32_t cnt = ls[nb - 1] + lh[nb - 1];
    const int64_t tile = a.tile0 + g;
    const int64_t base = tile * kPartTile;
    for (uint32_t j = threadIdx.x; j < cnt; j += THR) {
        if constexpr (N4) {
            __builtin_nontemporal_store(s_r32[j], reinterpret_cast<uint32_t*>(a.p1_key) + base + j);
            continue;
        }
        __builtin_nontemporal_store((int64_t)s.k[j], a.p1_key + base + j);  // read back a flush later
        if constexpr (NR) continue;
        if constexpr (C) {
            if constexpr (ACC) __builtin_nontemporal_store(s_v32[j], reinterpret_cast<int32_t*>(a.p1_a0) + base + j);
        } else {
            a.p1_a0[base + j] = s.a0[j];
            if constexpr (AV) a.p1_a1[base + j] = s.a1[j];
            a.p1_pos[base + j] = s.pos[j];
        }
    }
    for (int b = threadIdx.x; b < nb; b += THR) a.p1_row[tile * kPartBuckets + b] = desc_pack(ls[b], lh[b]);
    if constexpr ((C && ACC) || NR) {
        wide = wave_sum(wide);
        if (__lane_id() == 0 && wide) atomicAdd(&a.st->wide_vals, wide);
    }
}

template <int AGG, int FMT, bool GAP>
__global__ void __launch_bounds__(kPartThreads) GW_P1_ATTR k_rgn_p1(IngestArgs a) {
    constexpr bool C = FMT == kFmtCmp && cmp_agg<AGG>();
    constexpr bool NR = FMT == kFmtNar && cmp_agg<AGG>();
    constexpr bool AV = !C && !NR && (AGG == GW_AVG_I64 || AGG == GW_AVG_F64);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const TileLds s = tile_lds<AV>(smem);
    __shared__ uint32_t lh[kPartBuckets], ls[kPartBuckets];
    __shared__ unsigned long long s_occ;
    const int64_t g = blockIdx.x;
    const int64_t lo = g * kPartTile, hi = min(a.n, lo + (int64_t)kPartTile);
    if (g == 0 && threadIdx.x < 64 && a.st_host) publish_status_wave(a.st, a.st_host, a.st_seq);
    for (int b = threadIdx.x; b < kPartBuckets; b += blockDim.x) lh[b] = 0;
    if (threadIdx.x == 0) s_occ = 0;
    __syncthreads();
    unsigned long long late = 0, flags = 0, occ = 0;
    int64_t key[kPartItems], ts[kPartItems], val[kPartItems];
#pragma unroll
    for (int it = 0; it < kPartItems; ++it) {  // all loads in flight first
        const int64_t i = lo + it * kPartThreads + threadIdx.x;
        key[it] = 0; ts[it] = 0; val[it] = 0;
        if (i < hi) {
            if (a.pk_w && i >= a.pk_from) {  // a packed exchange word: 8 B instead of 24
                int64_t k, t, v;
                unpack_word(a.pk_g, __builtin_nontemporal_load(a.pk_w + (i - a.pk_from)), k, t, v);
                key[it] = k;
                ts[it] = t;
                if (a.val) val[it] = v;
            } else {
                key[it] = __builtin_nontemporal_load(a.key + i);  // read once: keep it out of the caches
                ts[it] = __builtin_nontemporal_load(a.ts + i);
                if (a.val) val[it] = __builtin_nontemporal_load(a.val + i);
            }
        }
    }
    p1_tile<AGG, FMT, GAP, kPartThreads, kPartItems>(a, g, lo, hi, key, ts, val, s, lh, ls, &s_occ, late, flags, occ);
    block_commit(a.st, late, 0, flags, occ);
}

// Plan, step 1 (block j = tile group [j*G, (j+1)*G)): transpose the group's descriptor
// rows into p2_desc[b][tile] and record each (bucket, group) block's size and rounds.
constexpr int kColBatch = 16;
__global__ void __launch_bounds__(256) k_rgn_plan1(IngestArgs a) {
    const int b = threadIdx.x;
    const int nb = 1 << a.d1_bits;
    if (b >= nb) return;
    const int64_t j = blockIdx.x;
    const int64_t t0 = j * a.p2_group, t1 = min(a.ntiles, t0 + (int64_t)a.p2_group);
    uint32_t size = 0;
    for (int64_t t = t0; t < t1; t += kColBatch) {
        uint32_t d[kColBatch];
#pragma unroll
        for (int q = 0; q < kColBatch; ++q) d[q] = a.p1_row[min(t + q, t1 - 1) * kPartBuckets + b];
#pragma unroll
        for (int q = 0; q < kColBatch; ++q) {
            if (t + q < t1) {
                a.p2_desc[(int64_t)b * a.ntiles + t + q] = d[q];
                size += d[q] & 0xffffu;
            }
        }
    }
    const int64_t k = (int64_t)b * a.ngroups + j;
    a.p2_off[k] = size;
    a.p2_roff[k] = (size + kPartTile - 1) / kPartTile;
}

// Plan, step 2 (block b = pass-1 bucket b): exclusive scans of its blocks' sizes and
// rounds over the groups (bucket-local); the bucket totals go to bk_off[b] / rbeg[b].
__global__ void __launch_bounds__(256) k_rgn_plan2(IngestArgs a) {
    __shared__ int64_t part[2][256];
    const int64_t b = blockIdx.x;
    const int64_t G = a.ngroups;
    const int64_t per = (G + 255) / 256;
    const int64_t lo = b * G + min(G, threadIdx.x * per), hi = b * G + min(G, (threadIdx.x + 1) * per);
    int64_t s0 = 0, s1 = 0;
    // loads in flight together: clamped (unconditional) addresses, values masked after
    for (int64_t k = lo; k < hi; k += kColBatch) {
        int64_t v0[kColBatch], v1[kColBatch];
#pragma unroll
        for (int q = 0; q < kColBatch; ++q) {
            const int64_t x = min(k + q, hi - 1);
            v0[q] = a.p2_off[x];
            v1[q] = a.p2_roff[x];
        }
#pragma unroll
        for (int q = 0; q < kColBatch; ++q) {
            if (k + q < hi) { s0 += v0[q]; s1 += v1[q]; }
        }
    }
    part[0][threadIdx.x] = s0;
    part[1][threadIdx.x] = s1;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const int64_t v0 = threadIdx.x >= (unsigned)o ? part[0][threadIdx.x - o] : 0;
        const int64_t v1 = threadIdx.x >= (unsigned)o ? part[1][threadIdx.x - o] : 0;
        __syncthreads();
        part[0][threadIdx.x] += v0;
        part[1][threadIdx.x] += v1;
        __syncthreads();
    }
    int64_t r0 = threadIdx.x ? part[0][threadIdx.x - 1] : 0, r1 = threadIdx.x ? part[1][threadIdx.x - 1] : 0;
    for (int64_t k = lo; k < hi; k += kColBatch) {
        int64_t v0[kColBatch], v1[kColBatch];
#pragma unroll
        for (int q = 0; q < kColBatch; ++q) {
            const int64_t x = min(k + q, hi - 1);
            v0[q] = a.p2_off[x];
            v1[q] = a.p2_roff[x];
        }
#pragma unroll
        for (int q = 0; q < kColBatch; ++q) {
            if (k + q >= hi) break;
            a.p2_off[k + q] = r0;
            a.p2_roff[k + q] = r1;
            r0 += v0[q];
            r1 += v1[q];
        }
    }
    if (threadIdx.x == 255) {
        a.bk_off[b] = part[0][255];
        a.rbeg[b] = part[1][255];
    }
}

// Plan, step 3 (one block): bucket totals -> bucket starts (records bk_off[], rounds
// rbeg[]), both exclusive with the grand total at [nb].
__global__ void __launch_bounds__(256) k_rgn_plan3(IngestArgs a) {
    __shared__ int64_t part[2][256];
    const int nb = 1 << a.d1_bits;
    const int b = threadIdx.x;
    const int64_t v0 = b < nb ? a.bk_off[b] : 0, v1 = b < nb ? a.rbeg[b] : 0;
    part[0][b] = v0;
    part[1][b] = v1;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const int64_t x0 = b >= o ? part[0][b - o] : 0, x1 = b >= o ? part[1][b - o] : 0;
        __syncthreads();
        part[0][b] += x0;
        part[1][b] += x1;
        __syncthreads();
    }
    if (b < nb) {
        a.bk_off[b] = part[0][b] - v0;
        a.rbeg[b] = part[1][b] - v1;
    }
    if (b == 255) {
        a.bk_off[nb] = part[0][255];
        a.rbeg[nb] = part[1][255];
    }
}

// P2: block (b1, j) -> rounds p2_roff[b1, j] ... of bucket b1, records at p2_off[b1, j].
template <int AGG, int FMT>
__global__ void __launch_bounds__(kPartThreads) k_rgn_p2(IngestArgs a) {
    constexpr bool C = FMT == kFmtCmp && cmp_agg<AGG>();
    constexpr bool NR = FMT == kFmtNar && cmp_agg<AGG>();
    constexpr bool N4 = NR && AGG == GW_COUNT;
    constexpr bool AV = !C && !NR && (AGG == GW_AVG_I64 || AGG == GW_AVG_F64);
    constexpr bool ACC = !(C && AGG == GW_COUNT);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const TileLds s = tile_lds<AV>(smem);
    int32_t* s_v32 = reinterpret_cast<int32_t*>(s.a0);
    uint32_t* s_r32 = reinterpret_cast<uint32_t*>(s.k);
    // pass-2 bucket: the region within the pass-1 bucket (pt_sub; C: of the hash word); narrow
    // two-pass flushes (nar2): (super-region, ring position)
    __shared__ uint32_t lh[kPartBuckets], ls[kPartBuckets];
    __shared__ uint32_t r_cnt[kMaxGroup], r_pre[kMaxGroup + 1], wsum[kPartThreads / 64];
    __shared__ int64_t r_src[kMaxGroup];
    const int64_t b1 = blockIdx.x / a.ngroups, j = blockIdx.x - b1 * a.ngroups;
    const int64_t t0 = j * a.p2_group;
    const int nt = (int)min((int64_t)a.p2_group, a.ntiles - t0);
    const int nb2 = a.nar2 ? (a.t.nsub >> a.sr_bits) << 3 : a.t.nsub;  // nar2: (super-region, ring position)
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
        const uint32_t d = a.p2_desc[b1 * a.ntiles + t0 + i];
        r_cnt[i] = d & 0xffffu;
        r_src[i] = (t0 + i) * kPartTile + (d >> 16);
    }
    __syncthreads();
    block_scan2(r_cnt, r_pre, nt, wsum);
    const uint32_t total = r_pre[nt];
    const float rpr = total ? (float)nt / (float)total : 0.f;  // run_near's guess (uniform)
    const int64_t k = b1 * a.ngroups + j;
    const int64_t out0 = a.bk_off[b1] + a.p2_off[k], rnd0 = a.rbeg[b1] + a.p2_roff[k];
    for (uint32_t e0 = 0; e0 < total; e0 += kPartTile) {
        const uint32_t e1 = min(total, e0 + (uint32_t)kPartTile);
        for (int b = threadIdx.x; b < kPartBuckets; b += blockDim.x) lh[b] = 0;
        __syncthreads();
        int64_t key[kPartItems], c0[kPartItems], c1[kPartItems];
        uint32_t pos[kPartItems], rank[kPartItems];
        int bk[kPartItems];
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            const uint32_t e = e0 + it * kPartThreads + threadIdx.x;
            key[it] = 0; c0[it] = 0; c1[it] = 0; pos[it] = 0;
            bk[it] = -1;
            if (e < e1) {
                const int i = run_near(r_pre, nt, e, rpr);
                const int64_t src = r_src[i] + (e - r_pre[i]);
                key[it] = N4 ? (int64_t)reinterpret_cast<const uint32_t*>(a.p1_key)[src] : a.p1_key[src];
                if constexpr (NR) {
                } else if constexpr (C) {
                    if constexpr (ACC) c0[it] = reinterpret_cast<const int32_t*>(a.p1_a0)[src];
                } else {
                    c0[it] = a.p1_a0[src];
                    if constexpr (AV) c1[it] = a.p1_a1[src];
                    pos[it] = a.p1_pos[src];
                }
                bk[it] = 0;
            }
        }
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            if (bk[it] < 0) continue;
            if constexpr (NR) {  // the key's hash gives its region
                const int64_t k = N4 ? nar_key32((uint32_t)key[it]) : nar_key((uint64_t)key[it]);
                bk[it] = pt_sub(a.t, slot_hash(k));
                if (a.nar2)
                    bk[it] = ((bk[it] >> a.sr_bits) << 3) |
                             (int)nar_pos(N4 ? (uint32_t)key[it] : (uint32_t)((uint64_t)key[it] >> 32));
            } else {
                bk[it] = pt_sub(a.t, C ? (uint64_t)key[it] : slot_hash(key[it]));
            }
            rank[it] = atomicAdd(&lh[bk[it]], 1u);
        }
        __syncthreads();
        scan_buckets(lh, ls, nb2);
        __syncthreads();
        const int64_t base = out0 + e0;
#pragma unroll
        for (int it = 0; it < kPartItems; ++it) {
            if (bk[it] < 0) continue;
            const uint32_t jj = ls[bk[it]] + rank[it];
            if constexpr (N4) {
                s_r32[jj] = (uint32_t)key[it];
                continue;
            }
            s.k[jj] = key[it];
            if constexpr (NR) continue;
            if constexpr (C) {
                if constexpr (ACC) s_v32[jj] = (int32_t)c0[it];
            } else {
                s.a0[jj] = c0[it];
                if constexpr (AV) s.a1[jj] = c1[it];
                s.pos[jj] = (uint8_t)pos[it];
            }
        }
        __syncthreads();
        const int64_t rnd = rnd0 + e0 / kPartTile;
        for (uint32_t jj = threadIdx.x; jj < e1 - e0; jj += blockDim.x) {
            if constexpr (N4) {
                __builtin_nontemporal_store(s_r32[jj], reinterpret_cast<uint32_t*>(a.e_key) + base + jj);
                continue;
            }
            __builtin_nontemporal_store((int64_t)s.k[jj], a.e_key + base + jj);
            if constexpr (NR) continue;
            if constexpr (C) {
                if constexpr (ACC) __builtin_nontemporal_store(s_v32[jj], reinterpret_cast<int32_t*>(a.e_a0) + base + jj);
            } else {
                a.e_a0[base + jj] = s.a0[jj];
                if constexpr (AV) a.e_a1[base + jj] = s.a1[jj];
                a.e_pos[base + jj] = s.pos[jj];
            }
        }
        for (int b = threadIdx.x; b < nb2; b += blockDim.x) a.r_row[rnd * kPartBuckets + b] = desc_pack(ls[b], lh[b]);
        if (threadIdx.x == 0) a.r_base[rnd] = base;
        __syncthreads();
    }
}

// apply: one workgroup per region; keys / mask / up to two active pane arrays in LDS
// Copy n int64 words (n even, both ends 16-B aligned) with 16-byte accesses.
__device__ __forceinline__ void copy_words(long long* __restrict__ d, const long long* __restrict__ s, int64_t n) {
    const int64_t n2 = n >> 1;
    const long2* s2 = reinterpret_cast<const long2*>(s);
    long2* d2 = reinterpret_cast<long2*>(d);
    for (int64_t w = threadIdx.x; w < n2; w += blockDim.x) d2[w] = s2[w];
}

#ifndef GW_APPLY_THREADS
#define GW_APPLY_THREADS 512
#endif
#ifndef GW_APPLY_GROUP
#define GW_APPLY_GROUP 4
#endif
#ifndef GW_APPLY_UNROLL
#define GW_APPLY_UNROLL 4
#endif
constexpr int kApplyThreads = GW_APPLY_THREADS;
constexpr int kApplyRuns = 256;  // run descriptors staged in LDS per step (<= blockDim)
constexpr int kApplyGroup = GW_APPLY_GROUP;   // consecutive runs a wave walks as one sequence
constexpr int kApplyUnroll = GW_APPLY_UNROLL;  // records per lane with their loads in flight together
constexpr int kApplyQ = 128;                   // per-wave queue of records that missed their home group
#ifndef GW_APPLY_FAST2
#define GW_APPLY_FAST2 0
#endif

template <int AGG, int FMT>
__global__ void __launch_bounds__(kApplyThreads) GW_APPLY_ATTR k_rgn_apply(IngestArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool M = uses_mask<AGG>();
    constexpr bool C = FMT == kFmtCmp && cmp_agg<AGG>();
    constexpr bool NR = FMT == kFmtNar && cmp_agg<AGG>();
    constexpr bool N4 = NR && AGG == GW_COUNT;
    constexpr bool AV = AGG == GW_AVG_I64 || AGG == GW_AVG_F64;  // (C: a1 = 1, not stored)
    constexpr bool ACC = !(C && AGG == GW_COUNT);
    __shared__ uint32_t r_cnt[kApplyRuns], r_src[kApplyRuns];  // buffer offsets < 2^32 (gw_runtime.cpp)
    const int64_t r = blockIdx.x;
    const int64_t S = pt_S(a.t);
    const int W = a.t.words;
    // this region's runs: rounds [rb, re) of its bucket, column col of their rows
    const int64_t bucket = r / a.t.nsub, col = r - bucket * a.t.nsub;
    const bool single = !a.two_pass;
    const int64_t rb = single ? 0 : a.rbeg[bucket], re = single ? a.ntiles : a.rbeg[bucket + 1];
    const int64_t ccol = single ? r : col;
    const uint32_t* rows = single ? a.p1_row : a.r_row;
    const int64_t* rk = single ? a.p1_key : a.e_key;
    const int64_t* ra0 = single ? a.p1_a0 : a.e_a0;
    const int64_t* ra1 = single ? a.p1_a1 : a.e_a1;
    const uint8_t* rpos = single ? a.p1_pos : a.e_pos;
    const int32_t* rv32 = reinterpret_cast<const int32_t*>(ra0);  // C: 32-bit values
    const uint32_t* rk32 = reinterpret_cast<const uint32_t*>(rk);  // N4: 4-byte records
    const uint64_t bucket_id = (uint64_t)bucket;                 // C: the hash's top d1 bits
    long long* lkeys = (long long*)smem;
    const int64_t MW = pt_mask_words(a.t);       // 0 unless M
    uint8_t* lmask = (uint8_t*)(lkeys + S);
    long long* lcell = lkeys + S + MW;           // [2][S][W]
    // per-wave queue of records that missed their home group (after the cells): hashes,
    // values (two words for averages), ring positions
    constexpr int QW = kApplyThreads / 64 * kApplyQ;
    unsigned char* qbase = reinterpret_cast<unsigned char*>(lcell + 2 * S * W);
    const int qoff = (threadIdx.x >> 6) * kApplyQ;
    uint64_t* qh = reinterpret_cast<uint64_t*>(qbase) + qoff;
    int64_t* qv0 = reinterpret_cast<int64_t*>(qbase + (size_t)QW * 8) + qoff;
    int64_t* qv1 = reinterpret_cast<int64_t*>(qbase + (size_t)QW * 16) + qoff;  // AV only
    uint8_t* qps = qbase + (size_t)QW * (AV ? 24 : 16) + qoff;
    int qn = 0;
    // dirty 128-B lines of the key array (S <= 2048: <= 128 lines)
    __shared__ uint32_t s_kdirty[4];
    // the (up to) two pane positions this flush touches
    const unsigned long long bocc = *(volatile unsigned long long*)a.batch_occ;
    const int act0 = bocc ? __ffsll((long long)bocc) - 1 : -1;
    const unsigned long long rest = bocc & (bocc - 1);
    const int act1 = rest ? __ffsll((long long)rest) - 1 : -1;
    int64_t* gkeys = pt_region(a.t, r);
    int64_t* gmask = gkeys + S;
    const int msh = a.t.mask_shift;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;

    // Prologue: the first block of run descriptors and the whole region state (keys +
    // mask, then each active pane array; a retired pane is the identity, not loaded) are
    // loaded in one memory round trip, then staged into LDS.
    const int nr0 = (int)min((int64_t)kApplyRuns, re - rb);
    uint32_t d0 = 0;
    int64_t base0 = 0;
    if ((int)threadIdx.x < nr0) {
        const int64_t rnd = rb + threadIdx.x;
        d0 = rows[rnd * kPartBuckets + ccol];
        base0 = single ? rnd * kPartTile : a.r_base[rnd];
    }
    const int64_t nkm = (S + MW) / 2, np = S * W / 2;  // in 16-B units
    const bool ld0 = act0 >= 0 && !((a.ring_fresh >> act0) & 1);
    const bool ld1 = act1 >= 0 && !((a.ring_fresh >> act1) & 1);
    const int64_t total2 = nkm + (act0 >= 0 ? np : 0) + (act1 >= 0 ? np : 0);
    const long2* gkm2 = reinterpret_cast<const long2*>(gkeys);
    const long2* gp0 = act0 >= 0 ? reinterpret_cast<const long2*>(pt_cell(a.t, r << a.t.log2S, act0)) : nullptr;
    const long2* gp1 = act1 >= 0 ? reinterpret_cast<const long2*>(pt_cell(a.t, r << a.t.log2S, act1)) : nullptr;
    const int64_t id0 = identity0(AGG);
    const long2 ident = W == 2 ? long2{id0, 0} : long2{id0, id0};
    // LDS-DMA (global_load_lds_dwordx4): each wave copies 1-KB pieces of the state
    // straight into LDS, 16 B per lane from a per-lane source, no VGPRs; a retired pane
    // is written as identities instead.
    long2* l2 = reinterpret_cast<long2*>(lkeys);
    for (int64_t w0 = (int64_t)wave * 64; w0 < total2; w0 += (int64_t)nw * 64) {
        const int64_t w = w0 + lane;
        const long2* src = nullptr;
        if (w < nkm) src = gkm2 + w;
        else if (w < nkm + np) { if (ld0) src = gp0 + (w - nkm); }
        else if (w < total2) { if (ld1) src = gp1 + (w - nkm - np); }
        if (src)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)(l2 + w0), 16, 0, 0);
        else if (w < total2)
            l2[w] = ident;
    }
    // uniform exit for a region without records (its first descriptor block is empty);
    // the barrier also waits for the LDS-DMA
    const int any = __syncthreads_or((int)(d0 & 0xffffu)) || (re - rb > kApplyRuns);
    if (!any) return;
    if constexpr (M) {  // a clear presence bit: the cell is the identity whatever it holds (a lazy
                        // fire retire, k_fire2); the loaded pane arrays are read after the run
                        // loop's first barrier
        for (int ai = 0; ai < 2 && a.stale; ++ai) {
            const int act = ai ? act1 : act0;
            if (!(ai ? ld1 : ld0)) continue;
            long long* lc = lcell + (int64_t)ai * S;
            for (int j = threadIdx.x; j < (int)S; j += blockDim.x)
                if (!((mask_get(lmask, j, msh) >> act) & 1)) lc[j] = id0;
        }
    }
    if ((int)threadIdx.x < nr0) {
        r_cnt[threadIdx.x] = d0 & 0xffffu;
        r_src[threadIdx.x] = (uint32_t)(base0 + (d0 >> 16));
    }
    if (threadIdx.x < 4) s_kdirty[threadIdx.x] = 0;
    // The LDS key array holds the keys' 64-bit hashes while the records apply (slot_hash is
    // a bijection; a free slot holds the hash of the empty marker, a key that never lives
    // in a normal slot): a compact record's word gives the hash without unhashing, and
    // only the dirty key lines are unhashed on the way back.  (The first barrier of the run
    // loop below orders this pass before any probe.)
    const long long kEmptyH = (long long)slot_hash(kEmptyKey);
    for (int j = threadIdx.x; j < (int)S; j += blockDim.x) lkeys[j] = (long long)slot_hash(lkeys[j]);
    unsigned long long ins = 0, flags = 0, spills = 0;
    // false: the region is full; the record stays in the buffer marked (pos | 0x80) and
    // k_rgn_collect parks it on the deferred list once the host has room for it
    auto apply_one = [&](uint64_t h, int64_t c0, int64_t c1, uint32_t pos) -> bool {
        const long long key = (long long)h;
        // Probe one 4-key group (32 B) per step: the first slot holding the key or
        // empty, in slot order, decides; an empty slot is claimed with a CAS (a lost race
        // re-reads the same group).
        // 32-bit LDS indices (S <= 2048 slots)
        const int Si = (int)S;
        int g0 = (int)pt_home(a.t, h);
        int found = -1;
        for (int p = 0; p < Si;) {
            const long2 k01 = *reinterpret_cast<const long2*>(&lkeys[g0]);
            const long2 k23 = *reinterpret_cast<const long2*>(&lkeys[g0 + 2]);
            const uint32_t hit = (uint32_t)(k01.x == key) | (uint32_t)(k01.y == key) << 1 |
                                 (uint32_t)(k23.x == key) << 2 | (uint32_t)(k23.y == key) << 3;
            const uint32_t emp = (uint32_t)(k01.x == kEmptyH) | (uint32_t)(k01.y == kEmptyH) << 1 |
                                 (uint32_t)(k23.x == kEmptyH) << 2 | (uint32_t)(k23.y == kEmptyH) << 3;
            const uint32_t m = hit | emp;
            if (m) {
                const int i = __ffs((int)m) - 1;
                const int j = g0 + i;
                if ((hit >> i) & 1) { found = j; break; }
                const unsigned long long prev = atomicCAS((unsigned long long*)&lkeys[j],
                                                          (unsigned long long)kEmptyH, (unsigned long long)key);
                if (prev == (unsigned long long)kEmptyH) {
                    found = j;
                    ins++;
                    atomicOr(&s_kdirty[j >> 9], 1u << ((j >> 4) & 31));
                    break;
                }
                if ((int64_t)prev == key) { found = j; break; }
                continue;  // another key took the slot: re-read this group
            }
            g0 = (g0 + kProbeGroup) & (Si - 1);
            p += kProbeGroup;
        }
        // Rare cases leave the record in the buffer (no global memory op here, so the
        // prefetched loads stay in flight): the region is full (the host grows the
        // table), or the record's pane is a third ring position in this flush.  The
        // spill pass below marks them for k_rgn_collect.
        if (found < 0) {
            flags |= GW_DF_TABLE_FULL;
            spills++;
            return false;
        }
        const int ai = (int)pos == act0 ? 0 : ((int)pos == act1 ? 1 : -1);
        if (ai < 0) {
            spills++;
            return false;
        }
        {
            long long* c = lcell + (ai * Si + found) * (AV ? 2 : 1);
            lds_cell_add<AGG>(c, c + (AV ? 1 : 0), c0, c1);
        }
        if constexpr (M) {  // presence bit: a non-returning LDS OR (the mask is written back whole)
            const uint32_t bit = ((uint32_t)found << (msh + 3)) + pos;
            atomicOr((uint32_t*)lmask + (bit >> 5), 1u << (bit & 31));
        }
        return true;
    };

    // Records: a wave takes kApplyGroup consecutive runs and walks their records as one
    // flattened sequence, kApplyUnroll records per lane per step; the loads of the next
    // step are issued before the current step is applied (one step of software
    // pipelining), so a wave always has a step of loads in flight.
    struct Grp {
        uint32_t pre[kApplyGroup + 1];
        uint32_t src[kApplyGroup];
    };
    struct Step {
        int64_t key[kApplyUnroll], v0[kApplyUnroll], v1[kApplyUnroll];
        uint8_t ps[kApplyUnroll];
        bool ok[kApplyUnroll];
    };
    for (int64_t c0r = rb; c0r < re; c0r += kApplyRuns) {
        const int nr = (int)min((int64_t)kApplyRuns, re - c0r);
        if (c0r != rb) {
            __syncthreads();  // previous block's descriptors fully consumed
            for (int i = threadIdx.x; i < nr; i += blockDim.x) {
                const int64_t rnd = c0r + i;
                const uint32_t d = rows[rnd * kPartBuckets + ccol];
                r_cnt[i] = d & 0xffffu;
                r_src[i] = (uint32_t)((single ? rnd * kPartTile : a.r_base[rnd]) + (d >> 16));
            }
        }
        __syncthreads();  // descriptors (and, first time, the region state) in LDS
        auto load_grp = [&](int i0, Grp& g) {
            g.pre[0] = 0;
#pragma unroll
            for (int u = 0; u < kApplyGroup; ++u) {
                const int i = i0 + u;
                g.pre[u + 1] = g.pre[u] + (i < nr ? r_cnt[i] : 0u);
                g.src[u] = i < nr ? r_src[i] : 0u;
            }
        };
        auto load_step = [&](const Grp& g, uint32_t k, Step& s, bool live) {
            const uint32_t tot = live ? g.pre[kApplyGroup] : 0u;
#pragma unroll
            for (int q = 0; q < kApplyUnroll; ++q) {
                const uint32_t e = k + q * 64 + lane;
                s.ok[q] = e < tot;
                uint32_t sb = g.src[0], sp = 0;  // static indices only: no scratch
#pragma unroll
                for (int w = 1; w < kApplyGroup; ++w) {
                    if (e >= g.pre[w]) { sb = g.src[w]; sp = g.pre[w]; }
                }
                // unconditional loads (an idle lane reads record 0): no branch around them,
                // so the compiler can count them and wait for exactly the ones it needs
                const uint32_t x = s.ok[q] ? sb + (e - sp) : 0u;
                s.key[q] = N4 ? (int64_t)rk32[x] : rk[x];
                s.v1[q] = 1;
                if constexpr (NR) {
                    s.v0[q] = 1;  // decoded in apply_step
                    s.ps[q] = 0;
                } else if constexpr (C) {
                    s.v0[q] = ACC ? (int64_t)rv32[x] : 1;
                    s.ps[q] = 0;  // in the word
                } else {
                    s.v0[q] = ra0[x];
                    if constexpr (AV) s.v1[q] = ra1[x];
                    s.ps[q] = rpos[x];
                }
            }
        };
        // next non-empty step after (i0, k) (k = ~0u: the first one), wave-uniform
        auto advance = [&](int& i0, uint32_t& k, Grp& g) -> bool {
            k = k == ~0u ? 0u : k + 64 * kApplyUnroll;
            while (i0 < nr && k >= g.pre[kApplyGroup]) {
                i0 += nw * kApplyGroup;
                k = 0;
                if (i0 < nr) load_grp(i0, g);
            }
            return i0 < nr;
        };
        int i0 = wave * kApplyGroup;
        uint32_t k = ~0u;
        Grp g;
        if (i0 < nr) load_grp(i0, g);
        // Two step buffers used in turn (no register copy of a step whose loads are still
        // in flight, which would wait for them): while one step is applied, the other's
        // loads are outstanding.  The loads are issued unconditionally, past the end as
        // well, so the compiler can count the outstanding ones on every path.
        // Fast path first: every record's home group (4 hashes, 32 B) is read with all the
        // step's LDS loads in flight together; a record whose key sits in its home group and
        // whose pane is active -- nearly all of them once the keys are in -- adds at once.
        // The rest (an insert, a key displaced beyond its group, a spill) take the generic
        // probe.  The table never holds an empty slot before a key in the key's probe order,
        // so a key found in its home group is exactly the slot the generic probe would pick.
        // Records whose key is not in its home group (an insert, a displaced key, a spill) go
        // to the wave's queue in LDS instead of probing at once: one lane's probe would hold
        // the whole wave.  64 at a time the wave probes them with every lane busy.
        auto q_push = [&](bool p, uint64_t hh, int64_t c0, int64_t c1, uint32_t pos) {
            const uint64_t bal = __ballot(p);
            if (p) {
                const int at = qn + __popcll(bal & ((1ull << lane) - 1ull));
                qh[at] = hh;
                qv0[at] = c0;
                if constexpr (AV) qv1[at] = c1;
                qps[at] = (uint8_t)pos;
            }
            qn += __popcll(bal);
            if (qn >= 64) {
                const int at = qn - 64 + lane;
                apply_one(qh[at], qv0[at], AV ? qv1[at] : 1, qps[at]);
                qn -= 64;
            }
        };
        auto apply_step = [&](const Step& c) {
            uint64_t h[kApplyUnroll];
            uint32_t ps[kApplyUnroll];
            int g[kApplyUnroll];
            long2 ka[kApplyUnroll], kb[kApplyUnroll];
            int64_t v0[kApplyUnroll];
#pragma unroll
            for (int q = 0; q < kApplyUnroll; ++q) {
                v0[q] = c.v0[q];
                if constexpr (NR) {
                    const uint64_t r = (uint64_t)c.key[q];
                    h[q] = slot_hash(N4 ? nar_key32((uint32_t)r) : nar_key(r));
                    ps[q] = nar_pos(N4 ? (uint32_t)r : (uint32_t)(r >> 32));
                    if constexpr (!N4) v0[q] = nar_val(r);
                } else if constexpr (C) {
                    h[q] = cmp_hash((uint64_t)c.key[q], bucket_id, a.d1_bits);
                    ps[q] = cmp_pos((uint64_t)c.key[q], a.d1_bits);
                } else {
                    h[q] = slot_hash(c.key[q]);
                    ps[q] = c.ps[q];
                }
                g[q] = (int)pt_home(a.t, h[q]);
            }
#pragma unroll
            for (int q = 0; q < kApplyUnroll; ++q) {
                ka[q] = *reinterpret_cast<const long2*>(&lkeys[g[q]]);
                kb[q] = *reinterpret_cast<const long2*>(&lkeys[g[q] + 2]);
            }
#if GW_APPLY_FAST2
            // a key displaced past its full home group is most often in the next group: read
            // it too (only where some lane needs it) before falling back to the queue
#pragma unroll
            for (int q = 0; q < kApplyUnroll; ++q) {
                const long long key = (long long)h[q];
                const bool hit = ka[q].x == key || ka[q].y == key || kb[q].x == key || kb[q].y == key;
                const bool full = ka[q].x != kEmptyH && ka[q].y != kEmptyH && kb[q].x != kEmptyH && kb[q].y != kEmptyH;
                const bool nxt = c.ok[q] && !hit && full;
                if (__any(nxt)) {
                    if (nxt) {
                        const int g2 = (g[q] + kProbeGroup) & ((int)S - 1);
                        const long2 na = *reinterpret_cast<const long2*>(&lkeys[g2]);
                        const long2 nb = *reinterpret_cast<const long2*>(&lkeys[g2 + 2]);
                        if (na.x == key || na.y == key || nb.x == key || nb.y == key) {
                            g[q] = g2;
                            ka[q] = na;
                            kb[q] = nb;
                        }
                    }
                }
            }
#endif
#pragma unroll
            for (int q = 0; q < kApplyUnroll; ++q) {
                bool fast = false;
                if (c.ok[q]) {
                    const long long key = (long long)h[q];
                    const int i = ka[q].x == key ? 0 : ka[q].y == key ? 1 : kb[q].x == key ? 2 : kb[q].y == key ? 3 : -1;
                    const int ai = (int)ps[q] == act0 ? 0 : ((int)ps[q] == act1 ? 1 : -1);
                    fast = i >= 0 && ai >= 0;
                    if (fast) {
                        const int found = g[q] + i;
                        long long* cl = lcell + (ai * (int)S + found) * (AV ? 2 : 1);
                        lds_cell_add<AGG>(cl, cl + (AV ? 1 : 0), v0[q], c.v1[q]);
                        if constexpr (M) {
                            const uint32_t bit = ((uint32_t)found << (msh + 3)) + ps[q];
                            atomicOr((uint32_t*)lmask + (bit >> 5), 1u << (bit & 31));
                        }
                    }
                }
                q_push(c.ok[q] && !fast, h[q], v0[q], c.v1[q], ps[q]);  // the wave is converged here
            }
        };
        Step sa, sb;
        bool live = advance(i0, k, g);
        load_step(g, k, sa, live);
        while (live) {
            live = advance(i0, k, g);
            load_step(g, k, sb, live);
            apply_step(sa);
            if (!live) break;
            live = advance(i0, k, g);
            load_step(g, k, sa, live);
            apply_step(sb);
        }
        if (lane < qn) apply_one(qh[lane], qv0[lane], AV ? qv1[lane] : 1, qps[lane]);  // the rest of the queue
        qn = 0;
    }
    // Spill pass (only in regions that had a spill): the final LDS key table says which
    // records were not applied: their key is absent (the region was full; no slot ever
    // frees up) or their ring position is not an active one.  Mark them (pos | 0x80).
    if (__syncthreads_or(spills != 0)) {
        unsigned long long marked = 0;
        for (int64_t c0r = rb; c0r < re; c0r += kApplyRuns) {
            const int nr = (int)min((int64_t)kApplyRuns, re - c0r);
            __syncthreads();
            for (int i = threadIdx.x; i < nr; i += blockDim.x) {
                const int64_t rnd = c0r + i;
                const uint32_t d = rows[rnd * kPartBuckets + ccol];
                r_cnt[i] = d & 0xffffu;
                r_src[i] = (uint32_t)((single ? rnd * kPartTile : a.r_base[rnd]) + (d >> 16));
            }
            __syncthreads();
            for (int i = wave; i < nr; i += nw) {
                for (uint32_t k = lane; k < r_cnt[i]; k += 64) {
                    const uint32_t x = r_src[i] + k;
                    int64_t key = N4 ? (int64_t)rk32[x] : rk[x];
                    uint32_t pos;
                    uint64_t h;
                    if constexpr (NR) {
                        const uint64_t r = (uint64_t)key;
                        h = slot_hash(N4 ? nar_key32((uint32_t)r) : nar_key(r));
                        pos = nar_pos(N4 ? (uint32_t)r : (uint32_t)(r >> 32));
                    } else if constexpr (C) {
                        h = cmp_hash((uint64_t)key, bucket_id, a.d1_bits);
                        pos = cmp_pos((uint64_t)key, a.d1_bits);
                    } else {
                        pos = rpos[x];
                        h = slot_hash(key);
                    }
                    bool present = false;
                    int64_t g0 = pt_home(a.t, h);
                    for (int64_t p = 0; p < S; ++p) {
                        const long long kk = lkeys[g0];
                        if (kk == (long long)h) { present = true; break; }
                        if (kk == kEmptyH) break;
                        g0 = (g0 + 1) & (S - 1);
                    }
                    if (!present || ((int)pos != act0 && (int)pos != act1)) {
                        if constexpr (N4) const_cast<uint32_t*>(rk32)[x] = rk32[x] | kNarSpill;
                        else if constexpr (NR) const_cast<int64_t*>(rk)[x] = (int64_t)((uint64_t)rk[x] | ((uint64_t)kNarSpill << 32));
                        else if constexpr (C) const_cast<int64_t*>(rk)[x] = (int64_t)((uint64_t)rk[x] | kCmpSpill);
                        else const_cast<uint8_t*>(rpos)[x] = (uint8_t)(pos | 0x80u);
                        marked++;
                    }
                }
            }
        }
        spills = marked;
    }
    __syncthreads();
    // write back: dirty 128-B lines of keys / mask, every line of the active pane arrays
    {
        const long2* sk = reinterpret_cast<const long2*>(lkeys);
        long2* dk = reinterpret_cast<long2*>(gkeys);
        for (int64_t w = threadIdx.x; w < S / 2; w += blockDim.x) {
            const int64_t line = w >> 3;
            if (s_kdirty[line >> 5] & (1u << (line & 31))) {
                const long2 v = sk[w];
                dk[w] = long2{slot_unhash((uint64_t)v.x), slot_unhash((uint64_t)v.y)};
            }
        }
    }
    if constexpr (M) copy_words((long long*)gmask, (const long long*)lmask, MW);
    for (int ai = 0; ai < 2; ++ai) {
        const int p = ai ? act1 : act0;
        if (p < 0) continue;
        copy_words((long long*)pt_cell(a.t, r << a.t.log2S, p), lcell + (int64_t)ai * S * W, S * W);
    }
    spills = wave_sum(spills);
    if (__lane_id() == 0 && spills) atomicAdd(&a.st->spills, spills);
    block_commit(a.st, 0, ins, flags, 0);
}

// ---------------------------------------------------------------------------
// Narrow two-pass apply (a.nar2, k_rgn_apply_nar): one workgroup per super-region of
// F = 2^sr_bits probe regions (F * S slots, consecutive in memory).  P2 wrote each round's
// records of a super-region grouped by ring position, so the workgroup applies one ring
// position after another with ONE pane's cells in LDS, while the keys (as 32-bit values:
// narrow keys are below 2^32 - 2) and the presence mask stay in LDS throughout.  Against
// k_rgn_apply: 4 + 1 + 8 B of LDS per slot instead of 8 + 1 + 16, so F = 2 regions per
// workgroup (runs F times longer, F times fewer workgroups and state round trips); a probe
// group is one 16-B LDS read; no hash pass over the keys on the way in or out; any number of
// ring positions per flush (no spill for a third one).
// ---------------------------------------------------------------------------
constexpr uint32_t kK32Empty = 0xffffffffu;    // a free slot
constexpr uint32_t kK32Foreign = 0xfffffffeu;  // a slot holding a key no narrow record carries
constexpr int kNarMaxF = 4;
constexpr int kNarMaxSlots = kNarMaxF * 2048;
constexpr int kNarLoadU = 4;  // 16-B state loads per thread in flight together
#ifndef GW_NAR_DEPTH
#define GW_NAR_DEPTH 2  // record steps whose loads are in flight (2: one ahead of the applied one)
#endif

__device__ __forceinline__ uint32_t k32_of(int64_t k) {
    return k == kEmptyKey ? kK32Empty : ((uint64_t)k < (uint64_t)kK32Foreign ? (uint32_t)k : kK32Foreign);
}

// STALE: cells behind clear presence bits may hold stale values (lazy fire retires, FireArgs::
// lazy_retire) and are staged as the identity; without it the staging is a plain copy.
template <int AGG, bool STALE>
__global__ void __launch_bounds__(kApplyThreads) GW_APPLY_ATTR k_rgn_apply_nar(IngestArgs a) {
    if constexpr (!cmp_agg<AGG>()) {
        return;
    } else {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool M = uses_mask<AGG>();
    constexpr bool N4 = AGG == GW_COUNT;
    constexpr int W = AGG == GW_AVG_I64 ? 2 : 1;
    __shared__ uint32_t r_cnt[kApplyRuns], r_src[kApplyRuns];
    __shared__ uint32_t s_kdirty[kNarMaxSlots / 16 / 32];  // dirty 128-B lines of the int64 key array
    __shared__ uint32_t s_pos;                              // ring positions holding records
    const int F = 1 << a.sr_bits;
    const int S = (int)pt_S(a.t), FS = F * S;
    const int l2S = a.t.log2S;
    const int64_t ncol = a.t.nsub >> a.sr_bits;  // super-regions per bucket
    const int64_t sr = blockIdx.x;
    const int64_t bucket = sr / ncol, col = sr - bucket * ncol;
    // the runs of this super-region: this flush's rounds (list 0) and the rounds of the
    // previous flush that carried ring positions (list 1, positions c_mask)
    const int64_t rb0 = a.cur_empty ? 0 : a.rbeg[bucket], re0 = a.cur_empty ? 0 : a.rbeg[bucket + 1];
    const int64_t rb1 = a.c_mask ? a.c_rbeg[bucket] : 0, re1 = a.c_mask ? a.c_rbeg[bucket + 1] : 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t* lkeys = reinterpret_cast<uint32_t*>(smem);                     // [FS]
    uint8_t* lmask = reinterpret_cast<uint8_t*>(lkeys + FS);                  // [FS] (M)
    long long* lcell = reinterpret_cast<long long*>(lmask + (M ? FS : 0));   // [FS][W]
    uint32_t* qk = reinterpret_cast<uint32_t*>(lcell + (int64_t)FS * W) + wave * kApplyQ;
    int32_t* qv = reinterpret_cast<int32_t*>(lcell + (int64_t)FS * W) + nw * kApplyQ + wave * kApplyQ;
    int qn = 0;
    const unsigned long long cur_pos = a.cur_empty ? 0ull : (*(volatile unsigned long long*)a.batch_occ) & a.apply_mask;
    // the region of hash h within the super-region: the low sr_bits of its region within the bucket (pt_sub)
    struct List {
        const uint32_t* rows;
        const int64_t* rbase;
        const uint64_t* rk;
        const uint32_t* rk32;
        int64_t rb, re;
        unsigned long long pos;  // ring positions this list contributes
    };
    // two named lists picked by a uniform select (an array indexed by the loop variable would
    // live in scratch memory)
    const List list0{a.r_row, a.r_base, reinterpret_cast<const uint64_t*>(a.e_key),
                     reinterpret_cast<const uint32_t*>(a.e_key), rb0, re0, cur_pos & 0xffull};
    const List list1{a.c_r_row, a.c_r_base, reinterpret_cast<const uint64_t*>(a.c_key),
                     reinterpret_cast<const uint32_t*>(a.c_key), rb1, re1, a.c_mask & 0xffull};

    // which ring positions hold records of this super-region (a region without any skips
    // the state round trip)
    if (threadIdx.x == 0) s_pos = 0;
    for (int i = threadIdx.x; i < kNarMaxSlots / 16 / 32; i += blockDim.x) s_kdirty[i] = 0;
    __syncthreads();
    {
        uint32_t any = 0;
        for (int l = 0; l < 2; ++l) {
            const List L = l ? list1 : list0;
            for (int64_t rnd = L.rb + threadIdx.x; rnd < L.re; rnd += blockDim.x)
                for (unsigned long long pm = L.pos; pm; pm &= pm - 1) {
                    const int p = __ffsll((long long)pm) - 1;
                    if (L.rows[rnd * kPartBuckets + ((col << 3) | p)] & 0xffffu) any |= 1u << p;
                }
        }
        any = (uint32_t)wave_ior(any);
        if (lane == 0 && any) atomicOr(&s_pos, any);
    }
    __syncthreads();
    const uint32_t pmask = s_pos;
    if (!pmask) return;  // uniform

    // keys (int64 in HBM -> 32-bit in LDS) and presence masks of the F regions
    {
        const int nk2 = FS / 2, nm16 = M ? FS / 16 : 0, tot = nk2 + nm16;
        for (int w0 = threadIdx.x; w0 < tot; w0 += kNarLoadU * blockDim.x) {
            long2 v[kNarLoadU];
#pragma unroll
            for (int u = 0; u < kNarLoadU; ++u) {
                const int w = w0 + u * blockDim.x;
                v[u] = long2{0, 0};
                if (w < nk2) {
                    const int d = w >> (l2S - 1), j = w & (S / 2 - 1);
                    v[u] = reinterpret_cast<const long2*>(pt_region(a.t, sr * F + d))[j];
                } else if (w < tot) {
                    const int wm_ = w - nk2, d = wm_ >> (l2S - 4), j = wm_ & (S / 16 - 1);
                    v[u] = reinterpret_cast<const long2*>(pt_mask_base(a.t, sr * F + d))[j];
                }
            }
#pragma unroll
            for (int u = 0; u < kNarLoadU; ++u) {
                const int w = w0 + u * blockDim.x;
                if (w < nk2) {
                    reinterpret_cast<uint2*>(lkeys)[w] = uint2{k32_of(v[u].x), k32_of(v[u].y)};
                } else if (w < tot) {
                    reinterpret_cast<long2*>(lmask)[w - nk2] = v[u];
                }
            }
        }
    }
    unsigned long long ins = 0, flags = 0, spills = 0;

    // Probe for key k (its hash h) in its region: one 4-key group per step, the first slot
    // holding k or free decides; a free slot is claimed by CAS (a lost race re-reads the
    // group).  Returns the slot in the super-region or -1 (the region is full).
    auto probe_insert = [&](uint32_t k, uint64_t h) -> int {
        const int d = F > 1 ? (int)(pt_sub(a.t, h) & (F - 1)) : 0;
        uint32_t* kd = lkeys + d * S;
        int g0 = (int)(h & (uint64_t)(S - 1) & ~(uint64_t)(kProbeGroup - 1));
        for (int p = 0; p < S;) {
            const uint4 kk = *reinterpret_cast<const uint4*>(kd + g0);
            const uint32_t hit = (uint32_t)(kk.x == k) | (uint32_t)(kk.y == k) << 1 | (uint32_t)(kk.z == k) << 2 |
                                 (uint32_t)(kk.w == k) << 3;
            const uint32_t emp = (uint32_t)(kk.x == kK32Empty) | (uint32_t)(kk.y == kK32Empty) << 1 |
                                 (uint32_t)(kk.z == kK32Empty) << 2 | (uint32_t)(kk.w == kK32Empty) << 3;
            const uint32_t m = hit | emp;
            if (m) {
                const int i = __ffs((int)m) - 1;
                const int j = g0 + i;
                if ((hit >> i) & 1) return d * S + j;
                const uint32_t prev = atomicCAS(kd + j, kK32Empty, k);
                if (prev == kK32Empty) {
                    ins++;
                    const int line = (d * S + j) >> 4;
                    atomicOr(&s_kdirty[line >> 5], 1u << (line & 31));
                    return d * S + j;
                }
                if (prev == k) return d * S + j;
                continue;  // another key took the slot: re-read this group
            }
            g0 = (g0 + kProbeGroup) & (S - 1);
            p += kProbeGroup;
        }
        return -1;
    };
    auto cell_add = [&](int slot, int64_t v, uint32_t bit) {
        long long* c = lcell + (int64_t)slot * W;
        lds_cell_add<AGG>(c, c + (W - 1), v, 1);
        if constexpr (M) atomicOr(reinterpret_cast<uint32_t*>(lmask) + (slot >> 2), bit << ((slot & 3) * 8));
    };

    struct Grp {
        uint32_t pre[kApplyGroup + 1];
        uint32_t src[kApplyGroup];
    };
    struct Step {
        uint64_t r[kApplyUnroll];
        bool ok[kApplyUnroll];
    };
    const long long id0 = identity0(AGG);
    const long2 ident = W == 2 ? long2{id0, 0} : long2{id0, id0};
    for (uint32_t pm = pmask; pm; pm &= pm - 1) {
        const int p = __ffs((int)pm) - 1;
        const uint32_t pbit = 1u << p;
        const int64_t ccol = (col << 3) | p;
        __syncthreads();  // the previous position's write-back has read the cells
        {  // this position's pane (an untouched one holds identities)
            const bool fresh = (a.ring_fresh >> p) & 1;
            const int per = S * W / 2, lper = l2S - 1 + (W == 2), tot = FS * W / 2;
            long2* l2 = reinterpret_cast<long2*>(lcell);
            for (int w0 = threadIdx.x; w0 < tot; w0 += kNarLoadU * blockDim.x) {
                long2 v[kNarLoadU];
                uint32_t mb[kNarLoadU];
#pragma unroll
                for (int u = 0; u < kNarLoadU; ++u) {
                    const int w = w0 + u * blockDim.x;
                    v[u] = ident;
                    mb[u] = ~0u;
                    if (w < tot && !fresh) {
                        const int d = w >> lper;
                        v[u] = reinterpret_cast<const long2*>(pt_cell(a.t, (sr * F + d) << l2S, p))[w - d * per];
                        // a clear presence bit: the cell is the identity whatever it holds (a lazy fire
                        // retire, k_fire2); one byte of mask per slot (ring <= 8), slots 2w, 2w + 1.  The
                        // mask's LDS reads are issued here, beside the cells' loads: read where they are
                        // used, each was a dependent LDS round trip per pair (Q7's apply 335 -> 540 us
                        // per flush, profiles/r6/q7/)
                        if constexpr (M && STALE) mb[u] = reinterpret_cast<const uint16_t*>(lmask)[w];
                    }
                }
#pragma unroll
                for (int u = 0; u < kNarLoadU; ++u) {
                    const int w = w0 + u * blockDim.x;
                    if (w >= tot) continue;
                    if constexpr (M && STALE) {
                        if (!((mb[u] >> p) & 1)) v[u].x = id0;
                        if (!((mb[u] >> (8 + p)) & 1)) v[u].y = id0;
                    }
                    l2[w] = v[u];
                }
            }
        }
        for (int l = 0; l < 2; ++l) {
            const List L = l ? list1 : list0;
            if (!((L.pos >> p) & 1)) continue;  // uniform
            const uint64_t* rk = L.rk;
            const uint32_t* rk32 = L.rk32;
            for (int64_t c0r = L.rb; c0r < L.re; c0r += kApplyRuns) {
                const int nr = (int)min((int64_t)kApplyRuns, L.re - c0r);
                __syncthreads();  // the cells are in; the previous block's descriptors consumed
                for (int i = threadIdx.x; i < nr; i += blockDim.x) {
                    const int64_t rnd = c0r + i;
                    const uint32_t d = L.rows[rnd * kPartBuckets + ccol];
                    r_cnt[i] = d & 0xffffu;
                    r_src[i] = (uint32_t)(L.rbase[rnd] + (d >> 16));
                }
                __syncthreads();
                auto load_grp = [&](int i0, Grp& g) {
                    g.pre[0] = 0;
#pragma unroll
                    for (int u = 0; u < kApplyGroup; ++u) {
                        const int i = i0 + u;
                        g.pre[u + 1] = g.pre[u] + (i < nr ? r_cnt[i] : 0u);
                        g.src[u] = i < nr ? r_src[i] : 0u;
                    }
                };
                auto load_step = [&](const Grp& g, uint32_t k, Step& st, bool live) {
                    const uint32_t tot = live ? g.pre[kApplyGroup] : 0u;
#pragma unroll
                    for (int q = 0; q < kApplyUnroll; ++q) {
                        const uint32_t e = k + q * 64 + lane;
                        st.ok[q] = e < tot;
                        uint32_t sb = g.src[0], sp = 0;
#pragma unroll
                        for (int w = 1; w < kApplyGroup; ++w) {
                            if (e >= g.pre[w]) { sb = g.src[w]; sp = g.pre[w]; }
                        }
                        const uint32_t x = st.ok[q] ? sb + (e - sp) : 0u;  // unconditional loads
                        st.r[q] = N4 ? (uint64_t)rk32[x] : rk[x];
                    }
                };
                auto advance = [&](int& i0, uint32_t& k, Grp& g) -> bool {
                    k = k == ~0u ? 0u : k + 64 * kApplyUnroll;
                    while (i0 < nr && k >= g.pre[kApplyGroup]) {
                        i0 += nw * kApplyGroup;
                        k = 0;
                        if (i0 < nr) load_grp(i0, g);
                    }
                    return i0 < nr;
                };
                // a record whose key is not in its home group waits in the wave's queue; 64 at a
                // time the wave probes them with every lane busy
                auto q_push = [&](bool pu, uint32_t kk, int32_t vv) {
                    const uint64_t bal = __ballot(pu);
                    if (pu) {
                        const int at = qn + __popcll(bal & ((1ull << lane) - 1ull));
                        qk[at] = kk;
                        qv[at] = vv;
                    }
                    qn += __popcll(bal);
                    if (qn >= 64) {
                        const int at = qn - 64 + lane;
                        const uint32_t k2 = qk[at];
                        const int s2 = probe_insert(k2, slot_hash((int64_t)k2));
                        if (s2 >= 0) cell_add(s2, qv[at], pbit);
                        else { flags |= GW_DF_TABLE_FULL; spills++; }
                        qn -= 64;
                    }
                };
                auto apply_step = [&](const Step& c) {
                    uint32_t kq[kApplyUnroll];
                    int32_t vq[kApplyUnroll];
                    int hq[kApplyUnroll];
                    uint4 ka[kApplyUnroll];
#pragma unroll
                    for (int q = 0; q < kApplyUnroll; ++q) {
                        const uint64_t r = c.r[q];
                        kq[q] = N4 ? (uint32_t)(r >> 4) : (uint32_t)r;
                        vq[q] = N4 ? 1 : (int32_t)(uint32_t)(r >> 32) >> 4;
                        const uint64_t h = slot_hash((int64_t)kq[q]);
                        const int d = F > 1 ? (int)(pt_sub(a.t, h) & (F - 1)) : 0;
                        hq[q] = d * S + (int)(h & (uint64_t)(S - 1) & ~(uint64_t)(kProbeGroup - 1));
                    }
#pragma unroll
                    for (int q = 0; q < kApplyUnroll; ++q) ka[q] = *reinterpret_cast<const uint4*>(lkeys + hq[q]);
#pragma unroll
                    for (int q = 0; q < kApplyUnroll; ++q) {
                        const uint32_t k = kq[q];
                        const int i = ka[q].x == k ? 0 : ka[q].y == k ? 1 : ka[q].z == k ? 2 : ka[q].w == k ? 3 : -1;
                        const bool fast = c.ok[q] && i >= 0;
                        if (fast) cell_add(hq[q] + i, vq[q], pbit);
                        q_push(c.ok[q] && !fast, k, vq[q]);  // the wave is converged here
                    }
                };
                int i0 = wave * kApplyGroup;
                uint32_t k = ~0u;
                Grp g;
                if (i0 < nr) load_grp(i0, g);
#if GW_NAR_DEPTH == 3
                // three step buffers in turn: two steps' loads in flight while one is applied
                // (advance() keeps returning false once the runs are exhausted)
                Step s0, s1, s2;
                bool v0 = advance(i0, k, g);
                load_step(g, k, s0, v0);
                bool v1 = advance(i0, k, g);
                load_step(g, k, s1, v1);
                while (v0) {
                    const bool v2 = advance(i0, k, g);
                    load_step(g, k, s2, v2);
                    apply_step(s0);
                    if (!v1) break;
                    v0 = advance(i0, k, g);
                    load_step(g, k, s0, v0);
                    apply_step(s1);
                    if (!v2) break;
                    v1 = advance(i0, k, g);
                    load_step(g, k, s1, v1);
                    apply_step(s2);
                }
#else
                Step sa, sb;
                bool live = advance(i0, k, g);
                load_step(g, k, sa, live);
                while (live) {
                    live = advance(i0, k, g);
                    load_step(g, k, sb, live);
                    apply_step(sa);
                    if (!live) break;
                    live = advance(i0, k, g);
                    load_step(g, k, sa, live);
                    apply_step(sb);
                }
#endif
                if (lane < qn) {  // the rest of the queue
                    const uint32_t k2 = qk[lane];
                    const int s2 = probe_insert(k2, slot_hash((int64_t)k2));
                    if (s2 >= 0) cell_add(s2, qv[lane], pbit);
                    else { flags |= GW_DF_TABLE_FULL; spills++; }
                }
                qn = 0;
            }
        }
        __syncthreads();
        {  // write back this position's pane
            const int per = S * W / 2, lper = l2S - 1 + (W == 2), tot = FS * W / 2;
            const long2* l2 = reinterpret_cast<const long2*>(lcell);
            for (int w = threadIdx.x; w < tot; w += blockDim.x) {
                const int d = w >> lper;
                reinterpret_cast<long2*>(pt_cell(a.t, (sr * F + d) << l2S, p))[w - d * per] = l2[w];
            }
        }
    }
    // Spill pass (only after a region filled up): records whose key is absent from the final
    // key table were not applied; mark them for k_rgn_collect_nar2.
    if (__syncthreads_or(spills != 0)) {
        unsigned long long marked = 0;
        for (int l = 0; l < 2; ++l) {
            const List L = l ? list1 : list0;
            for (unsigned long long pm = L.pos & pmask; pm; pm &= pm - 1) {
                const int p = __ffsll((long long)pm) - 1;
                const int64_t ccol = (col << 3) | p;
                for (int64_t rnd = L.rb + wave; rnd < L.re; rnd += nw) {
                    const uint32_t d = L.rows[rnd * kPartBuckets + ccol];
                    const int64_t src = L.rbase[rnd] + (d >> 16);
                    for (uint32_t k = lane; k < (d & 0xffffu); k += 64) {
                        const uint64_t r = N4 ? (uint64_t)L.rk32[src + k] : L.rk[src + k];
                        const uint32_t kk = N4 ? (uint32_t)(r >> 4) : (uint32_t)r;
                        const uint64_t h = slot_hash((int64_t)kk);
                        const int dd = F > 1 ? (int)(pt_sub(a.t, h) & (F - 1)) : 0;
                        int j = (int)(h & (uint64_t)(S - 1) & ~(uint64_t)(kProbeGroup - 1));
                        bool present = false;
                        for (int q = 0; q < S; ++q) {
                            const uint32_t x = lkeys[dd * S + j];
                            if (x == kk) { present = true; break; }
                            if (x == kK32Empty) break;
                            j = (j + 1) & (S - 1);
                        }
                        if (!present) {
                            if constexpr (N4) const_cast<uint32_t*>(L.rk32)[src + k] = (uint32_t)r | kNarSpill;
                            else const_cast<uint64_t*>(L.rk)[src + k] = r | ((uint64_t)kNarSpill << 32);
                            marked++;
                        }
                    }
                }
            }
        }
        spills = marked;
    }
    __syncthreads();
    // write back: the masks whole, the keys of dirty lines (a foreign slot never changes)
    if constexpr (M) {
        const int per = S / 16, lper = l2S - 4;
        for (int w = threadIdx.x; w < FS / 16; w += blockDim.x) {
            const int d = w >> lper;
            reinterpret_cast<long2*>(pt_mask_base(a.t, sr * F + d))[w - d * per] = reinterpret_cast<const long2*>(lmask)[w];
        }
    }
    for (int j = threadIdx.x; j < FS; j += blockDim.x) {
        const int line = j >> 4;
        if ((s_kdirty[line >> 5] >> (line & 31)) & 1u) {
            const uint32_t k = lkeys[j];
            if (k != kK32Foreign) {
                const int d = j >> l2S;
                pt_region(a.t, sr * F + d)[j - d * S] = k == kK32Empty ? kEmptyKey : (int64_t)k;
            }
        }
    }
    spills = wave_sum(spills);
    if (__lane_id() == 0 && spills) atomicAdd(&a.st->spills, spills);
    block_commit(a.st, 0, ins, flags, 0);
    }
}

// Spilled narrow records of a nar2 flush: one linear pass over the P2 output.
template <int AGG>
__global__ void __launch_bounds__(256) k_rgn_collect_nar2(IngestArgs a) {
    constexpr bool N4 = AGG == GW_COUNT;
    // this flush's P2 output, then (blockIdx.y == 1) the carried output it applied from
    const bool carry = blockIdx.y == 1;
    if (carry ? !a.c_mask : a.cur_empty) return;
    const int nb1 = 1 << a.d1_bits;
    const int64_t n = carry ? a.c_rbeg[kPartBuckets + 1 + nb1] : a.bk_off[nb1];
    int64_t* rk = carry ? a.c_key : a.e_key;
    uint32_t* rk32 = reinterpret_cast<uint32_t*>(rk);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        bool spill = false;
        int64_t key = 0, pane = 0, c0 = 0;
        if (i < n) {
            const uint64_t w = N4 ? (uint64_t)rk32[i] : (uint64_t)rk[i];
            const uint32_t lo = N4 ? (uint32_t)w : (uint32_t)(w >> 32);
            if (nar_spilled(lo)) {
                spill = true;
                if (N4) rk32[i] = (uint32_t)w & ~kNarSpill;
                else rk[i] = (int64_t)(w & ~((uint64_t)kNarSpill << 32));
                key = N4 ? nar_key32((uint32_t)w) : nar_key(w);
                c0 = N4 ? 1 : nar_val(w);
                const int64_t rel = ((int64_t)nar_pos(lo) - a.b_pos + a.t.ring) % a.t.ring;
                pane = a.p_late + (int64_t)a.delta + rel;
            }
        }
        defer_write(a, spill, key, pane, c0, 1);
    }
}

// The same for compact records: the spill mark is bit 63 of the word, and the key comes
// back from the hash, whose top bits are the record's bucket -- so one workgroup per
// region walks the region's runs as the apply does.
template <int AGG>
__global__ void __launch_bounds__(256) k_rgn_collect_cmp(IngestArgs a) {
    constexpr bool ACC = AGG != GW_COUNT;
    const int64_t r = blockIdx.x;
    const int64_t bucket = r / a.t.nsub, col = r - bucket * a.t.nsub;
    const bool single = !a.two_pass;
    const int64_t rb = single ? 0 : a.rbeg[bucket], re = single ? a.ntiles : a.rbeg[bucket + 1];
    const int64_t ccol = single ? r : col;
    const uint32_t* rows = single ? a.p1_row : a.r_row;
    int64_t* rk = single ? a.p1_key : a.e_key;
    const int32_t* rv32 = reinterpret_cast<const int32_t*>(single ? a.p1_a0 : a.e_a0);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int64_t rnd = rb + wave; rnd < re; rnd += nw) {  // a wave per run: uniform loop bounds
        const uint32_t d = rows[rnd * kPartBuckets + ccol];
        const uint32_t cnt = d & 0xffffu;
        const int64_t src = (single ? rnd * kPartTile : a.r_base[rnd]) + (d >> 16);
        for (uint32_t k0 = 0; k0 < cnt; k0 += 64) {
            const uint32_t k = k0 + lane;
            bool spill = false;
            int64_t key = 0, pane = 0, c0 = 0;
            if (k < cnt) {
                const uint64_t w = (uint64_t)rk[src + k];
                if (w & kCmpSpill) {
                    spill = true;
                    rk[src + k] = (int64_t)(w & ~kCmpSpill);
                    key = slot_unhash(cmp_hash(w, (uint64_t)bucket, a.d1_bits));
                    const uint32_t pos = cmp_pos(w, a.d1_bits);
                    c0 = ACC ? (int64_t)rv32[src + k] : 1;
                    const int64_t rel = ((int64_t)pos - a.b_pos + a.t.ring) % a.t.ring;
                    pane = a.p_late + (int64_t)a.delta + rel;
                }
            }
            defer_write(a, spill, key, pane, c0, 1);
        }
    }
}

// The same for narrow records (spill bit next to the ring position; the key is the record's).
template <int AGG>
__global__ void __launch_bounds__(256) k_rgn_collect_nar(IngestArgs a) {
    constexpr bool N4 = AGG == GW_COUNT;
    const int64_t r = blockIdx.x;
    const int64_t bucket = r / a.t.nsub, col = r - bucket * a.t.nsub;
    const bool single = !a.two_pass;
    const int64_t rb = single ? 0 : a.rbeg[bucket], re = single ? a.ntiles : a.rbeg[bucket + 1];
    const int64_t ccol = single ? r : col;
    const uint32_t* rows = single ? a.p1_row : a.r_row;
    int64_t* rk = single ? a.p1_key : a.e_key;
    uint32_t* rk32 = reinterpret_cast<uint32_t*>(rk);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int64_t rnd = rb + wave; rnd < re; rnd += nw) {  // a wave per run: uniform loop bounds
        const uint32_t d = rows[rnd * kPartBuckets + ccol];
        const uint32_t cnt = d & 0xffffu;
        const int64_t src = (single ? rnd * kPartTile : a.r_base[rnd]) + (d >> 16);
        for (uint32_t k0 = 0; k0 < cnt; k0 += 64) {
            const uint32_t k = k0 + lane;
            bool spill = false;
            int64_t key = 0, pane = 0, c0 = 0;
            if (k < cnt) {
                const uint64_t w = N4 ? (uint64_t)rk32[src + k] : (uint64_t)rk[src + k];
                const uint32_t lo = N4 ? (uint32_t)w : (uint32_t)(w >> 32);
                if (nar_spilled(lo)) {
                    spill = true;
                    if (N4) rk32[src + k] = (uint32_t)w & ~kNarSpill;
                    else rk[src + k] = (int64_t)(w & ~((uint64_t)kNarSpill << 32));
                    key = N4 ? nar_key32((uint32_t)w) : nar_key(w);
                    c0 = N4 ? 1 : nar_val(w);
                    const int64_t rel = ((int64_t)nar_pos(lo) - a.b_pos + a.t.ring) % a.t.ring;
                    pane = a.p_late + (int64_t)a.delta + rel;
                }
            }
            defer_write(a, spill, key, pane, c0, 1);
        }
    }
}

// After a flush that filled regions: park every spilled record (pos | 0x80 in the
// buffer) on the deferred list; the host has made room for st->spills entries.
template <int AGG>
__global__ void __launch_bounds__(256) k_rgn_collect(IngestArgs a) {
    const bool single = !a.two_pass;
    const int nb = 1 << a.d1_bits;
    const int64_t n = single ? a.ntiles * kPartTile : a.bk_off[nb];
    const int64_t* rk = single ? a.p1_key : a.e_key;
    const int64_t* ra0 = single ? a.p1_a0 : a.e_a0;
    const int64_t* ra1 = single ? a.p1_a1 : a.e_a1;
    uint8_t* rpos = single ? a.p1_pos : a.e_pos;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < n; base += stride) {
        const int64_t i = base + threadIdx.x;
        bool spill = false;
        int64_t key = 0, pane = 0, c0 = 0, c1 = 0;
        if (i < n) {
            bool valid = true;
            if (single) {  // tile-local records: [0, start + count of the last bucket)
                const uint32_t d = a.p1_row[(i / kPartTile) * kPartBuckets + nb - 1];
                valid = (i % kPartTile) < (int64_t)((d >> 16) + (d & 0xffffu));
            }
            const uint32_t pos = rpos[i];
            if (valid && (pos & 0x80u)) {
                spill = true;
                rpos[i] = (uint8_t)(pos & 0x7fu);
                key = rk[i];
                c0 = ra0[i];
                c1 = ra1 ? ra1[i] : 1;
                const int64_t rel = ((int64_t)(pos & 0x7fu) - a.b_pos + a.t.ring) % a.t.ring;
                pane = a.p_late + (int64_t)a.delta + rel;
            }
        }
        defer_write(a, spill, key, pane, c0, c1);
    }
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

// ---------------------------------------------------------------------------
// Allowed lateness > 0: rows of late records for fired, not yet cleaned windows
// ---------------------------------------------------------------------------
// Reference: WindowOperator.processElement :408-446 adds the record to every window
// that is not late (cleanup time > watermark) and, because EventTimeTrigger.onElement
// returns FIRE for a window whose max timestamp <= watermark (EventTimeTrigger.java:
// 37-45), emits that window's contents right away; under PurgingTrigger the contents
// are purged after each emission, so a late record's row holds that record alone.
// Here the late records of one watermark interval are sorted by (key, arrival); one
// thread per key walks them in arrival order, keeping a per-pane running fold on top
// of the table's panes, and emits one row per (record, re-firing window).  The records
// are merged into the table afterwards (k_merge_deferred).
__device__ __forceinline__ int64_t pt_find_ro(const PaneTable& t, int64_t key) {
    if (key == kEmptyKey) return t.cap;
    const uint64_t h = slot_hash(key);
    const int64_t S = pt_S(t);
    const int64_t r = pt_key_region(t, h);
    const int64_t* keys = pt_region(t, r);
    int64_t j = pt_home(t, h);
    const int lim = S < kMaxProbe ? (int)S : kMaxProbe;
    for (int p = 0; p < lim; ++p) {
        const int64_t k = keys[j];
        if (k == key) return (r << t.log2S) + j;
        if (k == kEmptyKey) return -1;
        j = (j + 1) & (S - 1);
    }
    return -1;
}



constexpr int kRefireThreads = 64;
template <int AGG>
__global__ void __launch_bounds__(kRefireThreads) k_refire(RefireArgs a) {
    // this interval's late records per ring position, per thread: LDS [R][threads] x 2
    extern __shared__ int64_t rf_lds[];
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int64_t key = a.rf_key[a.order[i]];
    if (i > 0 && a.rf_key[a.order[i - 1]] == key) return;  // not the first record of its key
    const int R = a.t.ring;
    const int W = a.t.words;
    const int64_t id0 = identity0(AGG);
    const int64_t g = pt_find_ro(a.t, key);
    const uint64_t mask = g >= 0 ? presence<AGG>(a.t, g) : 0;
    const int64_t oh = (a.ov.head && g >= 0) ? a.ov.head[g] : -1;
    int64_t* run0 = rf_lds + threadIdx.x;  // run0[q * kRefireThreads]
    int64_t* run1 = rf_lds + R * kRefireThreads + threadIdx.x;
    for (int q = 0; q < R; ++q) { run0[q * kRefireThreads] = id0; run1[q * kRefireThreads] = 0; }
    for (int64_t j = i; j < a.n && a.rf_key[a.order[j]] == key; ++j) {
        const uint32_t e = a.order[j];
        const int64_t p = a.rf_pane[e], c0 = a.rf_a0[e], c1 = a.rf_a1[e];
        const bool in_ring = p >= a.b && p - a.b < R;
        int pos = 0;
        if (in_ring) {
            pos = a.b_pos + (int)(p - a.b);
            if (pos >= R) pos -= R;
            fold_cell(AGG, run0[pos * kRefireThreads], run1[pos * kRefireThreads], c0, c1);
        }
        const int64_t k0 = max(a.k_lo, floor_div_d(p - a.np, a.m) + 1), k1 = min(a.k_hi, floor_div_d(p, a.m));
        for (int64_t k = k0; k <= k1; ++k) {
            int64_t r0 = id0, r1 = 0;
            if (a.purging) {
                fold_cell(AGG, r0, r1, c0, c1);
            } else {
                if (oh >= 0) {  // restored state of this fired window
                    for (int64_t q = oh; q < a.ov.n && a.ov.key[q] == key && a.ov.k[q] <= k; ++q)
                        if (a.ov.k[q] == k && !(a.ov.flags[q] & kOvDead)) fold_cell(AGG, r0, r1, a.ov.a0[q], a.ov.a1[q]);
                }
                for (int64_t q = k * a.m; q < k * a.m + a.np; ++q) {
                    if (q < a.b || q - a.b >= R) continue;  // outside the ring: no data
                    int qp = a.b_pos + (int)(q - a.b);
                    if (qp >= R) qp -= R;
                    if ((mask >> qp) & 1) {
                        const int64_t* c = pt_cell(a.t, g, qp);
                        fold_cell(AGG, r0, r1, c[0], W == 2 ? c[1] : 0);
                    }
                    fold_cell(AGG, r0, r1, run0[qp * kRefireThreads], run1[qp * kRefireThreads]);
                }
            }
            const unsigned long long o = atomicAdd(&a.st->rows, 1ull);
            const int64_t st = a.offset + k * a.slide;
            a.o_key[o] = key;
            a.o_start[o] = st;
            a.o_end[o] = st + a.size;
            a.o_res[o] = cell_result(AGG, r0, r1);
        }
    }
}

__global__ void __launch_bounds__(256) k_refire_keys(int mode, const int64_t* src, int64_t base, uint64_t* k,
                                                     uint32_t* v, int64_t n) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mode == 0) {
        k[i] = (uint64_t)(src[i] - base);
        v[i] = (uint32_t)i;
    } else {
        k[i] = (uint64_t)src[v[i]];
    }
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
    if (a.guarded && *(volatile unsigned long long*)&a.st->fire_skip) return;  // uniform: set before this launch
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
        int64_t oi = -1;  // this key's next restored-window entry
        if (live) {
            key = *pt_key(a.t, g);
            mask = presence<AGG>(a.t, g);
            if (a.ov.head) oi = a.ov.head[g];
        }
        for (int w = 0; w < a.nwin; ++w) {
            const bool flush = rs.cnt + blockDim.x > kRowStage;  // uniform: read before any append
            __syncthreads();
            if (flush) stage_flush(rs, &a.st->rows, a.o_key, a.o_start, a.o_end, a.o_res);
            uint64_t m = mask & a.wmask[w];
            bool ov_hit = false;
            int64_t o0 = 0, o1 = 0;
            if (oi >= 0) {  // restored state of (key, window): fires with its timer or with new records
                const int64_t kk = a.k0 + w;
                while (oi < a.ov.n && a.ov.key[oi] == key && a.ov.k[oi] < kk) ++oi;
                if (oi < a.ov.n && a.ov.key[oi] == key && a.ov.k[oi] == kk) {
                    const uint32_t f = a.ov.flags[oi];
                    if (!(f & kOvDead) && (m || (f & kOvTimer))) {
                        ov_hit = true;
                        o0 = a.ov.a0[oi];
                        o1 = a.ov.a1[oi];
                        a.ov.flags[oi] = a.ov.purge ? kOvDead : (f & ~kOvTimer);
                    }
                } else if (oi >= a.ov.n || a.ov.key[oi] != key) {
                    oi = -1;
                }
            }
            if (m || ov_hit) {
                int64_t r0 = id0, r1 = 0;
                while (m) {
                    const int pos = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    const int64_t* c = pt_cell(a.t, g, pos);
                    fold_cell(AGG, r0, r1, c[0], W == 2 ? c[1] : 0);
                }
                if (ov_hit) fold_cell(AGG, r0, r1, o0, o1);
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
                if (a.lazy_retire && g != a.t.cap) continue;  // as k_fire2
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

// Fire sweep, round 5 (k_fire2): the latency-hiding form of k_fire for passes without a
// restored-window overlay whose windows read at most 6 ring positions (Nexmark Q5: 5 of 6;
// tumbling: 1).  Every lane takes U slots per step and loads each slot's key, presence mask
// and the cells of the NP positions the pass reads -- unconditionally: the lines come in
// whole either way -- one step AHEAD of the step it folds, so a wave always has a step's
// loads in flight while it works.  Rows are compacted per wave with ballots; each wave
// reserves its rows in the workgroup's LDS stage with one LDS atomic per window and step
// (k_fire: one per row, and a barrier pair per window), and the stage goes out with one
// device atomic per kRowStage rows.  Same rows and retire as k_fire.
constexpr int kF2Threads = 256;
constexpr int kF2Stage = 2048;
template <int AGG, int NP, int U>
__global__ void __launch_bounds__(kF2Threads) k_fire2(FireArgs a) {
    if (a.guarded && *(volatile unsigned long long*)&a.st->fire_skip) return;  // uniform: set before this launch
    constexpr bool M = uses_mask<AGG>();
    constexpr bool AV = AGG == GW_AVG_I64 || AGG == GW_AVG_F64;
    __shared__ long long s_k[kF2Stage], s_r[kF2Stage];
    __shared__ uint8_t s_w[kF2Stage];
    __shared__ unsigned s_cnt;
    __shared__ unsigned long long s_base;
    const int64_t nslots = a.t.cap + 1;
    const int64_t id0 = identity0(AGG);
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) s_cnt = 0;
    if (blockIdx.x == 0 && threadIdx.x < kShards) atomicAnd(&a.st->sh[threadIdx.x].occ, ~a.rmask);
    uint64_t need = 0;
    for (int w = 0; w < a.nwin; ++w) need |= a.wmask[w];
    int posl[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        posl[q] = need ? __ffsll((long long)need) - 1 : posl[q > 0 ? q - 1 : 0];
        need &= need - 1;
    }
    const int64_t S = pt_S(a.t);
    const int64_t MW = pt_mask_words(a.t);
    const int ms = a.t.mask_shift;
    constexpr int64_t step = (int64_t)kF2Threads * U;
    const int64_t per = (nslots + gridDim.x - 1) / gridDim.x;
    const int64_t chunk = (per + step - 1) / step * step;
    const int64_t c0 = (int64_t)blockIdx.x * chunk, c1 = min(nslots, c0 + chunk);
    struct Buf {
        int64_t key[U];
        uint64_t mask[U];
        int64_t v0[U][NP];
        int64_t v1[U][AV ? NP : 1];
    };
    auto load = [&](Buf& b, int64_t base) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t g0 = base + u * kF2Threads + threadIdx.x;
            const int64_t g = g0 < c1 ? g0 : c1 - 1;  // unconditional: clamped into the chunk
            const int64_t* rg = pt_region(a.t, g >> a.t.log2S);
            const int64_t j = g & (S - 1);
            b.key[u] = rg[j];
            b.mask[u] = M ? mask_get((const uint8_t*)(rg + S), j, ms) : 0;
            const int64_t* cells = rg + S + MW;
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const int64_t* c = cells + ((int64_t)posl[q] * S + j) * (AV ? 2 : 1);
                b.v0[u][q] = c[0];
                if constexpr (AV) b.v1[u][q] = c[1];
            }
        }
    };
    auto flush = [&]() {  // every thread; ends with s_cnt == 0
        __syncthreads();
        const unsigned c = s_cnt;
        if (threadIdx.x == 0 && c) s_base = atomicAdd(&a.st->rows, (unsigned long long)c);
        __syncthreads();
        const unsigned long long b = s_base;
        for (unsigned j = threadIdx.x; j < c; j += kF2Threads) {
            const int64_t st = a.start0 + (int64_t)s_w[j] * a.slide;
            a.o_key[b + j] = s_k[j];
            a.o_start[b + j] = st;
            a.o_end[b + j] = st + a.size;
            a.o_res[b + j] = s_r[j];
        }
        __syncthreads();
        if (threadIdx.x == 0) s_cnt = 0;
        __syncthreads();
    };
    auto fold = [&](const Buf& b, int64_t base) {
        for (int w = 0; w < a.nwin; ++w) {
            const uint64_t wm = a.wmask[w];
            int64_t res[U];
            uint64_t bal[U];
            unsigned tot = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int64_t r0 = id0, r1 = 0;
                bool any = false;
#pragma unroll
                for (int q = 0; q < NP; ++q) {
                    const bool in = (wm >> posl[q]) & 1;
                    const bool pres = M ? ((b.mask[u] >> posl[q]) & 1) != 0 : (AV ? b.v1[u][q] : b.v0[u][q]) != 0;
                    if (in && pres) {
                        fold_cell(AGG, r0, r1, b.v0[u][q], AV ? b.v1[u][q] : 0);
                        any = true;
                    }
                }
                any = any && base + u * kF2Threads + threadIdx.x < c1;
                res[u] = cell_result(AGG, r0, r1);
                bal[u] = __ballot(any);
                tot += (unsigned)__popcll(bal[u]);
            }
            unsigned o = 0;
            if (lane == 0 && tot) o = atomicAdd(&s_cnt, tot);
            o = __shfl(o, 0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if ((bal[u] >> lane) & 1) {
                    const unsigned j = o + (unsigned)__popcll(bal[u] & ((1ull << lane) - 1ull));
                    s_k[j] = b.key[u];
                    s_r[j] = res[u];
                    s_w[j] = (uint8_t)w;
                }
                o += (unsigned)__popcll(bal[u]);
            }
        }
        if (a.rmask) {  // clearAllState of the panes no later window covers
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t g = base + u * kF2Threads + threadIdx.x;
                if (g >= c1) continue;
                int64_t* rg = pt_region(a.t, g >> a.t.log2S);
                const int64_t j = g & (S - 1);
                if constexpr (M) {
                    if (b.mask[u] & a.rmask) mask_put((uint8_t*)(rg + S), j, ms, b.mask[u] & ~a.rmask);
                }
                // presence-mask aggregates (lazy_retire): the clear bits are the retire; the
                // sentinel slot, which pass 1 adds into with device atomics, is reset for real
                if (M && a.lazy_retire && g != a.t.cap) continue;
                for (uint64_t m = a.rmask; m; m &= m - 1) {
                    const int pos = __ffsll((long long)m) - 1;
                    int64_t* c = rg + S + MW + ((int64_t)pos * S + j) * (AV ? 2 : 1);
                    c[0] = id0;
                    if constexpr (AV) c[1] = 0;
                }
            }
        }
        __syncthreads();  // every wave's rows of this step are staged
        if (s_cnt + (unsigned)(step * a.nwin) > (unsigned)kF2Stage) flush();  // uniform
    };
    __syncthreads();
    if (c0 < c1) {
        Buf A, B;
        load(A, c0);
        for (int64_t base = c0; base < c1; base += 2 * step) {
            const bool more = base + step < c1;  // uniform
            if (more) load(B, base + step);
            fold(A, base);
            if (!more) break;
            if (base + 2 * step < c1) load(A, base + 2 * step);
            fold(B, base + step);
        }
    }
    flush();
}

// Lazy retires (FireArgs::lazy_retire) made good: every cell of ring positions `pm` whose
// presence bit is clear becomes the identity.  Run before a kernel that adds into cells with
// device atomics (direct / pre-aggregation ingest, deferred merge); the region apply and every
// reader go by the presence bits and need no cleaning.
template <int AGG>
__global__ void __launch_bounds__(256) k_clean_stale(PaneTable t, uint64_t pm) {
    if constexpr (uses_mask<AGG>()) {
        const int64_t id0 = identity0(AGG);
        for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < t.cap; g += (int64_t)gridDim.x * blockDim.x) {
            const uint64_t m = pt_mask_get(t, g);
            for (uint64_t q = pm & ~m; q; q &= q - 1) pt_cell(t, g, __ffsll((long long)q) - 1)[0] = id0;
        }
    }
}

// One wave: the guard of a fire enqueued right behind a flush (gw_kernels.h FireGuard), over
// the status as the launches before it left it.
__global__ void __launch_bounds__(64) k_fire_guard(DevStatus* st, FireGuard g) {
    const int lane = threadIdx.x;
    unsigned long long flags = 0, used = 0;
    for (int i = lane; i < kShards; i += 64) {
        flags |= st->sh[i].flags;
        used += st->sh[i].ins;
    }
    flags = wave_ior(flags);
    used = wave_sum(used);
    if (lane == 0) {
        if (g.reset_rows) st->rows = 0;
        const unsigned long long rows = g.reset_rows ? 0ull : st->rows;
        const bool skip = st->spills != 0 || st->wide_vals != 0 ||
                          (flags & (GW_DF_TABLE_FULL | GW_DF_NO_TS | GW_DF_RANGE)) != 0 ||
                          st->n_deferred != g.expect_ndef ||
                          (int64_t)rows + g.nwin * ((int64_t)used + 1) > g.o_cap;
        st->fire_skip = skip ? 1ull : 0ull;
        st->fire_rows0 = rows;
    }
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

// Snapshot (gw_snapshot): every non-null pane cell of the table and every deferred entry
// whose key group lies in [kg_lo, kg_hi] -> (key, pane, a0, a1, kg) entries.
template <int AGG>
__global__ void __launch_bounds__(256) k_snap_collect(SnapArgs a) {
    const int64_t nslots = a.t.cap + 1;
    const int W = a.t.words;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t total = nslots + a.n_def;
    for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < total; base += stride) {
        const int64_t i = base + threadIdx.x;
        uint64_t m = 0;
        int64_t key = 0;
        int32_t kg = -1;
        bool def = false;
        if (i < nslots) {
            key = i == a.t.cap ? kEmptyKey : *pt_key(a.t, i);
            m = presence<AGG>(a.t, i) & a.occ;
        } else if (i < total) {
            key = a.d_key[i - nslots];
            def = true;
        }
        if (m || def) {
            kg = key_group_for_hash(java_long_hash(key), a.max_p);
            if (kg < a.kg_lo || kg > a.kg_hi) { m = 0; def = false; }
        }
        const unsigned cnt = def ? 1u : (unsigned)__popcll(m);
        unsigned long long off = wave_reserve_n(a.n_out, cnt);
        if (def) {
            const int64_t j = i - nslots;
            a.o_key[off] = key; a.o_pane[off] = a.d_pane[j]; a.o_a0[off] = a.d_a0[j]; a.o_a1[off] = a.d_a1[j];
            a.o_kg[off] = kg;
        }
        while (m) {
            const int pos = __ffsll((long long)m) - 1;
            m &= m - 1;
            const int64_t* c = pt_cell(a.t, i, pos);
            a.o_key[off] = key; a.o_pane[off] = a.pane_of_pos[pos];
            a.o_a0[off] = c[0]; a.o_a1[off] = W == 2 ? c[1] : 0;
            a.o_kg[off] = kg;
            off++;
        }
    }
}

// Restore: every overlay key gets a slot (inserted with no pane data) and head[slot] points at
// its first entry (entries sorted by key).
__global__ void __launch_bounds__(256) k_overlay_attach(PaneTable t, Overlay ov, int32_t* head, DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < ov.n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i > 0 && ov.key[i - 1] == ov.key[i]) continue;
        bool inserted;
        const int64_t g = pt_find_or_insert(t, ov.key[i], inserted);
        if (g < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        ins += inserted;
        head[g] = (int32_t)i;
    }
    block_commit(st, 0, ins, flags, 0);
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

hipError_t launch_table_init(const PaneTable& t, hipStream_t s) {
#define L(A) hipLaunchKernelGGL(k_table_init<A>, dim3(grid_for(t.cap + 1)), dim3(256), 0, s, t)
    GW_AGG_SWITCH(t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_ingest(const IngestArgs& a, int path, int unroll, hipStream_t s) {
    if (path == 1) {
        static int cus = 0;
        if (!cus) {
            int dev = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            cus = std::max(cus, 1);
        }
        static const int bpc = getenv("GW_PREAGG_BPC") ? std::max(1, atoi(getenv("GW_PREAGG_BPC"))) : 2;
        const int g = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)bpc * cus, (a.n + 2047) / 2048));
#define L(A) hipLaunchKernelGGL(k_ingest_preagg<A>, dim3(g), dim3(256), 0, s, a)
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

// A launch that stamps timing events with its own start / end when given them (e0 / e1 of
// launch_region_p1 / launch_region_flush / launch_fire), a plain launch otherwise.
#define GW_TLAUNCH(K, G, B, L, S, E0, E1, ...)                                \
    do {                                                                      \
        if ((E0) || (E1)) hipExtLaunchKernelGGL(K, G, B, L, S, E0, E1, 0, __VA_ARGS__); \
        else hipLaunchKernelGGL(K, G, B, L, S, __VA_ARGS__);                   \
    } while (0)

// A timed launch with no kernel to run: both events at this point of the stream (so they are
// valid and measure ~0).
static hipError_t record_empty(hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (e0) { const hipError_t e = hipEventRecord(e0, s); if (e != hipSuccess) return e; }
    if (e1) { const hipError_t e = hipEventRecord(e1, s); if (e != hipSuccess) return e; }
    return hipSuccess;
}

// Opt a kernel in to more than 64 KB of dynamic LDS (gfx950 has 160 KB per CU) once per
// size, not per launch: the attribute call costs host time on every ingest otherwise.
static void lds_opt_in(const void* f, size_t bytes) {
    static std::mutex mu;
    static std::vector<std::pair<const void*, size_t>> done;
    std::lock_guard<std::mutex> lock(mu);
    for (auto& d : done)
        if (d.first == f && d.second >= bytes) return;
    hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    done.emplace_back(f, bytes);
}

static size_t part_lds_bytes(const IngestArgs& a) {
    if (a.fmt == kFmtNar) return (size_t)kPartTile * (a.t.agg == GW_COUNT ? 4 : 8);
    if (a.fmt == kFmtCmp) return (size_t)kPartTile * 12;  // hash word + 32-bit value
    return (size_t)kPartTile * 8 * (a.t.words == 2 ? 3 : 2) + 2 * kPartTile;
}

int region_group(int d1_bits) {
    // P1 tiles per P2 workgroup: 7/4 of the pass-1 buckets, so a bucket's runs over a group
    // fill about two 4096-record rounds (one round per workgroup: flush 0.668 -> 0.653 ms at
    // the headline with two, 0.82 ms with half a round; GW_P2_GROUP overrides for experiments)
    static const int env = getenv("GW_P2_GROUP") ? atoi(getenv("GW_P2_GROUP")) : 0;
    if (env > 0) return std::min(kMaxGroup, env);
    return std::max(1, std::min(kMaxGroup, 7 * (1 << d1_bits) * 4096 / (4 * kPartTile)));
}

// Region path, P1 over one watermark batch: one block per 4096-record tile.
hipError_t launch_region_p1(const IngestArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const int64_t tiles = (a.n + kPartTile - 1) / kPartTile;
    if (tiles == 0) return record_empty(s, e0, e1);
    const size_t part_lds = part_lds_bytes(a);
    // beyond the 64 KB default: opt in (gfx950 has 160 KB of LDS per CU)
    // the gap test (size < slide) only in a variant of its own: it costs the hot pass ~3%
#define P1L(A, F, G)                                                                                            \
    lds_opt_in((const void*)k_rgn_p1<A, F, G>, part_lds);                                                      \
    GW_TLAUNCH((k_rgn_p1<A, F, G>), dim3((unsigned)tiles), dim3(kPartThreads), part_lds, s, e0, e1, a)
#define L(A)                                  \
    if (a.gap_size) {                         \
        P1L(A, kFmtWide, true);               \
    } else if (a.fmt == kFmtNar) {            \
        P1L(A, kFmtNar, false);               \
    } else if (a.fmt == kFmtCmp) {            \
        P1L(A, kFmtCmp, false);               \
    } else {                                  \
        P1L(A, kFmtWide, false);              \
    }
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
#undef P1L
    return hipGetLastError();
}

hipError_t launch_publish_status(const IngestArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_publish_status, dim3(1), dim3(256), 0, s, a.st, a.st_host, a.st_seq);
    return hipGetLastError();
}

// Region path, per flush over a.ntiles buffer tiles: plan + P2 (two-pass tables), then
// one workgroup per region applies its runs.
hipError_t launch_region_flush(const IngestArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const bool single = !a.two_pass;
    const size_t part_lds = part_lds_bytes(a);
    const int64_t S = pt_S(a.t);
    const size_t apply_lds = (size_t)(S + pt_mask_words(a.t)) * 8 + (size_t)2 * S * a.t.words * 8 +
                             (size_t)(kApplyThreads / 64) * kApplyQ * (a.t.words == 2 ? 25 : 17);  // + miss queues
    const int nb1 = 1 << a.d1_bits;
    if (a.ntiles == 0 && !(a.nar2 && a.c_mask)) return record_empty(s, e0, e1);
#define L2(A, CM)                                                                                               \
    lds_opt_in((const void*)k_rgn_p2<A, CM>, part_lds);                                                       \
    lds_opt_in((const void*)k_rgn_apply<A, CM>, apply_lds);                                                   \
    if (!single) {                                                                                              \
        GW_TLAUNCH(k_rgn_plan1, dim3((unsigned)a.ngroups), dim3(256), 0, s, e0, nullptr, a);                   \
        hipLaunchKernelGGL(k_rgn_plan2, dim3((unsigned)nb1), dim3(256), 0, s, a);                              \
        hipLaunchKernelGGL(k_rgn_plan3, dim3(1), dim3(256), 0, s, a);                                          \
        hipLaunchKernelGGL((k_rgn_p2<A, CM>), dim3((unsigned)(a.ngroups * nb1)), dim3(kPartThreads), part_lds, s, \
                           a);                                                                                  \
    }                                                                                                           \
    GW_TLAUNCH((k_rgn_apply<A, CM>), dim3((unsigned)a.t.nreg), dim3(kApplyThreads), apply_lds, s,               \
               single ? e0 : nullptr, e1, a)
#define L(A)                        \
    if (a.fmt == kFmtNar) {         \
        L2(A, kFmtNar);             \
    } else if (a.fmt == kFmtCmp) {  \
        L2(A, kFmtCmp);             \
    } else {                        \
        L2(A, kFmtWide);            \
    }
    if (a.fmt == kFmtNar && a.nar2) {
        const int F = 1 << a.sr_bits;
        const int64_t FS = (int64_t)F * S;
        const bool M = a.t.has_mask != 0;
        const size_t lds = (size_t)FS * 4 + (M ? (size_t)FS : 0) + (size_t)FS * a.t.words * 8 +
                           (size_t)(kApplyThreads / 64) * kApplyQ * 8;
#define LN(A)                                                                                                   \
    lds_opt_in((const void*)k_rgn_p2<A, kFmtNar>, part_lds);                                                   \
    lds_opt_in((const void*)k_rgn_apply_nar<A, true>, lds);                                                   \
    lds_opt_in((const void*)k_rgn_apply_nar<A, false>, lds);                                                  \
    if (!a.cur_empty) {                                                                                         \
        GW_TLAUNCH(k_rgn_plan1, dim3((unsigned)a.ngroups), dim3(256), 0, s, e0, nullptr, a);                   \
        hipLaunchKernelGGL(k_rgn_plan2, dim3((unsigned)nb1), dim3(256), 0, s, a);                              \
        hipLaunchKernelGGL(k_rgn_plan3, dim3(1), dim3(256), 0, s, a);                                          \
        hipLaunchKernelGGL((k_rgn_p2<A, kFmtNar>), dim3((unsigned)(a.ngroups * nb1)), dim3(kPartThreads), part_lds, \
                           s, a);                                                                               \
    }                                                                                                           \
    if (a.stale)                                                                                                \
        GW_TLAUNCH((k_rgn_apply_nar<A, true>), dim3((unsigned)(a.t.nreg >> a.sr_bits)), dim3(kApplyThreads), lds, \
                   s, a.cur_empty ? e0 : nullptr, e1, a);                                                       \
    else                                                                                                        \
        GW_TLAUNCH((k_rgn_apply_nar<A, false>), dim3((unsigned)(a.t.nreg >> a.sr_bits)), dim3(kApplyThreads),     \
                   lds, s, a.cur_empty ? e0 : nullptr, e1, a)
        GW_AGG_SWITCH(a.t.agg, LN);
#undef LN
        return hipGetLastError();
    }
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
#undef L2
    return hipGetLastError();
}

hipError_t launch_region_collect(const IngestArgs& a, hipStream_t s) {
    const int64_t n = a.ntiles * kPartTile;  // upper bound of the buffer's records
#define L(A)                                                                                         \
    if (a.fmt == kFmtNar && a.nar2)                                                                  \
        hipLaunchKernelGGL(k_rgn_collect_nar2<A>, dim3(grid_for(n), 2), dim3(256), 0, s, a);        \
    else if (a.fmt == kFmtNar)                                                                       \
        hipLaunchKernelGGL(k_rgn_collect_nar<A>, dim3((unsigned)a.t.nreg), dim3(256), 0, s, a);     \
    else if (a.fmt == kFmtCmp)                                                                       \
        hipLaunchKernelGGL(k_rgn_collect_cmp<A>, dim3((unsigned)a.t.nreg), dim3(256), 0, s, a);     \
    else                                                                                             \
        hipLaunchKernelGGL(k_rgn_collect<A>, dim3(grid_for(n)), dim3(256), 0, s, a)
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_merge_deferred(const MergeArgs& a, hipStream_t s) {
#define L(A) hipLaunchKernelGGL(k_merge_deferred<A>, dim3(grid_for(a.n)), dim3(256), 0, s, a)
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_refire(const RefireArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const size_t lds = (size_t)2 * a.t.ring * kRefireThreads * 8;
#define L(A) hipLaunchKernelGGL(k_refire<A>, dim3((unsigned)((a.n + kRefireThreads - 1) / kRefireThreads)), \
                                dim3(kRefireThreads), lds, s, a)
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_refire_keys(int mode, const int64_t* src, int64_t base, uint64_t* k, uint32_t* v, int64_t n,
                              hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_refire_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, mode, src, base, k, v, n);
    return hipGetLastError();
}

hipError_t launch_deferred_min(const int64_t* pane, int64_t n, DevStatus* st, hipStream_t s) {
    hipLaunchKernelGGL(k_deferred_min, dim3(grid_for(n)), dim3(256), 0, s, pane, n, st);
    return hipGetLastError();
}

hipError_t launch_fire(const FireArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    uint64_t need = 0;
    for (int w = 0; w < a.nwin; ++w) need |= a.wmask[w];
    const int npos = __builtin_popcountll(need);
    if (a.ov.head == nullptr && npos >= 1 && npos <= 6 && a.nwin <= 255 &&
        (int64_t)a.nwin * kF2Threads * 2 <= kF2Stage) {
        const bool av = a.t.agg == GW_AVG_I64 || a.t.agg == GW_AVG_F64;
        const int64_t tile = (int64_t)kF2Threads * (av ? 1 : 2);  // U slots per lane
        const int fg = (int)std::min<int64_t>(1024, std::max<int64_t>(1, (a.t.cap + 1 + tile - 1) / tile));
#define F2(A, NPV) \
    GW_TLAUNCH((k_fire2<A, NPV, (A == GW_AVG_I64 || A == GW_AVG_F64) ? 1 : 2>), dim3(fg), dim3(kF2Threads), 0, s, e0, e1, a)
#define L(A)                      \
    switch (npos) {               \
    case 1: F2(A, 1); break;      \
    case 2: F2(A, 2); break;      \
    case 3: F2(A, 3); break;      \
    case 4: F2(A, 4); break;      \
    case 5: F2(A, 5); break;      \
    default: F2(A, 6); break;     \
    }
        GW_AGG_SWITCH(a.t.agg, L);
#undef L
#undef F2
        return hipGetLastError();
    }
    const int fg = (int)std::min<int64_t>(1024, std::max<int64_t>(1, (a.t.cap + 1 + 255) / 256));
#define L(A) GW_TLAUNCH(k_fire<A>, dim3(fg), dim3(256), 0, s, e0, e1, a)
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_fire_guard(DevStatus* st, const FireGuard& g, hipStream_t s) {
    hipLaunchKernelGGL(k_fire_guard, dim3(1), dim3(64), 0, s, st, g);
    return hipGetLastError();
}

hipError_t launch_clean_stale(const PaneTable& t, uint64_t pmask, hipStream_t s) {
    if (!t.has_mask || !pmask) return hipSuccess;
#define L(A) hipLaunchKernelGGL(k_clean_stale<A>, dim3(grid_for(t.cap)), dim3(256), 0, s, t, pmask)
    GW_AGG_SWITCH(t.agg, L);
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

hipError_t launch_snap_collect(const SnapArgs& a, hipStream_t s) {
#define L(A) hipLaunchKernelGGL(k_snap_collect<A>, dim3(grid_for(a.t.cap + 1 + a.n_def)), dim3(256), 0, s, a)
    GW_AGG_SWITCH(a.t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_overlay_attach(const PaneTable& t, const Overlay& ov, int32_t* head, DevStatus* st, hipStream_t s) {
    if (ov.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_overlay_attach, dim3(grid_for(ov.n)), dim3(256), 0, s, t, ov, head, st);
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
