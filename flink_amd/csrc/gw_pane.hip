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
#include "gw_kernels.h"

#include <algorithm>

namespace gw {

template <int AGG>
__global__ void __launch_bounds__(256) k_table_init(TableView t) {
    const int64_t nslots = t.cap + 1;
    const int64_t id0 = identity0(AGG);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nslots;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t* s = slot_ptr(t, i);
        s[0] = kEmptyKey;
        s[1] = 0;
        for (int r = 0; r < t.ring; ++r) {
            s[2 + r * t.words] = id0;
            if (t.words == 2) s[3 + r * t.words] = 0;
        }
    }
}

template <int AGG>
__device__ __forceinline__ constexpr bool uses_mask() {
    return !(AGG == GW_COUNT || AGG == GW_AVG_I64 || AGG == GW_AVG_F64);
}

// Ring positions of a slot holding a non-null accumulator.  COUNT / AVG carry a
// count in the cell, so presence is `count != 0` and ingest never touches word 1;
// the other aggregates keep an explicit presence mask in word 1.
template <int AGG>
__device__ __forceinline__ uint64_t presence(const int64_t* s, int R, int W) {
    if constexpr (uses_mask<AGG>()) {
        return (uint64_t)s[1];
    } else {
        uint64_t m = 0;
        for (int r = 0; r < R; ++r)
            if (s[2 + r * W + (W - 1)] != 0) m |= 1ull << r;
        return m;
    }
}
__device__ __forceinline__ uint64_t presence_rt(const int64_t* s, const TableView& t) {
    if (t.agg == GW_COUNT || t.agg == GW_AVG_I64 || t.agg == GW_AVG_F64) {
        uint64_t m = 0;
        for (int r = 0; r < t.ring; ++r)
            if (s[2 + r * t.words + (t.words - 1)] != 0) m |= 1ull << r;
        return m;
    }
    return (uint64_t)s[1];
}

// Continue a linear probe from `idx` (the first slot was already read as `k0`).
__device__ __forceinline__ int64_t probe_from(const TableView& t, int64_t key, uint64_t idx, int64_t k0,
                                              bool& inserted) {
    inserted = false;
    const uint64_t mask = (uint64_t)t.cap - 1;
    int64_t k = k0;
    for (int p = 0; p < kMaxProbe; ++p) {
        int64_t* s = slot_ptr(t, (int64_t)idx);
        if (p) k = *(volatile int64_t*)s;
        if (k == key) return (int64_t)idx;
        if (k == kEmptyKey) {
            const unsigned long long prev = atomicCAS((unsigned long long*)s, (unsigned long long)kEmptyKey,
                                                      (unsigned long long)key);
            if (prev == (unsigned long long)kEmptyKey) { inserted = true; return (int64_t)idx; }
            if ((int64_t)prev == key) return (int64_t)idx;
        }
        idx = (idx + 1) & mask;
    }
    return -1;
}

// Direct path: one device-scope atomic RMW into the record's (slot, pane) cell, plus
// one presence-bit OR on the first touch of a (key, pane) for SUM/MIN/MAX.
// U records per thread per iteration: their first probes are issued back to back so
// each lane keeps U random 64-B line reads in flight (memory-level parallelism).
template <int AGG, int U>
__global__ void __launch_bounds__(256) k_ingest(IngestArgs a) {
    const int64_t tile = (int64_t)blockDim.x * U;
    const int64_t stride = (int64_t)gridDim.x * tile;
    unsigned long long late = 0, ins = 0, flags = 0, occ = 0;
    const uint64_t R = (uint64_t)a.t.ring;
    const uint64_t tmask = (uint64_t)a.t.cap - 1;
    const uint32_t W = (uint32_t)a.t.words;
    for (int64_t base = blockIdx.x * tile; base < a.n; base += stride) {
        int64_t key[U], c0[U], c1[U], pane[U], k0[U];
        uint64_t idx[U];
        uint32_t pos[U];
        int state[U];  // 0 skip, 1 in ring, 2 defer
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)u * blockDim.x + threadIdx.x;
            state[u] = 0;
            key[u] = 0; c0[u] = 0; c1[u] = 0; pane[u] = 0; pos[u] = 0;
            if (i < a.n) {
                key[u] = a.key[i];
                const int64_t ts = a.ts[i];
                const int64_t v = a.val ? a.val[i] : 0;
                if (ts == INT64_MIN) {
                    flags |= GW_DF_NO_TS;
                } else if (ts < a.t_late) {
                    if (a.late_exact) late++;
                    else flags |= GW_DF_RANGE;
                } else {
                    const uint64_t q = udiv64((uint64_t)ts - (uint64_t)a.t_late, a.div);
                    record_cell(AGG, v, c0[u], c1[u]);
                    const uint64_t rel = q - a.delta;
                    pane[u] = a.p_late + (int64_t)q;
                    if (q >= a.delta && rel < R) {
                        uint32_t p = (uint32_t)a.b_pos + (uint32_t)rel;
                        if (p >= R) p -= (uint32_t)R;
                        pos[u] = p;
                        state[u] = 1;
                    } else {
                        if (q > (uint64_t)(INT64_MAX - a.p_late)) flags |= GW_DF_RANGE;
                        state[u] = 2;
                    }
                }
            }
        }
        // first probes of all U records, issued together
#pragma unroll
        for (int u = 0; u < U; ++u) {
            idx[u] = key[u] == kEmptyKey ? (uint64_t)a.t.cap : (slot_hash(key[u]) & tmask);
            k0[u] = state[u] == 1 ? *(volatile int64_t*)slot_ptr(a.t, (int64_t)idx[u]) : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (state[u] != 1) continue;
            int64_t si;
            if (key[u] == kEmptyKey) {
                si = a.t.cap;  // sentinel slot of the key Long.MIN_VALUE
            } else {
                bool inserted;
                si = probe_from(a.t, key[u], idx[u], k0[u], inserted);
                ins += inserted;
            }
            if (si < 0) {
                flags |= GW_DF_TABLE_FULL;
                state[u] = 2;
                continue;
            }
            int64_t* s = slot_ptr(a.t, si);
            cell_atomic<AGG>(s + 2 + pos[u] * W, c0[u], c1[u]);
            const unsigned long long bit = 1ull << pos[u];
            if constexpr (uses_mask<AGG>()) {
                if (!(*(volatile unsigned long long*)(s + 1) & bit)) atomicOr((unsigned long long*)(s + 1), bit);
            }
            occ |= bit;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool defer = state[u] == 2;
            const unsigned long long off = wave_reserve(&a.st->n_deferred, defer);
            if (defer) {
                a.d_key[off] = key[u];
                a.d_pane[off] = pane[u];
                a.d_a0[off] = c0[u];
                a.d_a1[off] = c1[u];
            }
        }
    }
    block_commit(a.st, late, ins, flags, occ);
}

// LDS pre-aggregation path (low key cardinality per batch, e.g. YSB's 100 campaigns):
// records are combined per (slot, pane) cell in a 2048-entry LDS hash table with LDS
// atomics; each block then flushes one device atomic per distinct cell instead of one
// per record, removing the same-address atomic serialisation in HBM.
constexpr int kLdsCells = 2048;
constexpr int kPreaggItems = 8;  // records per thread per tile

template <int AGG>
__global__ void __launch_bounds__(256) k_ingest_preagg(IngestArgs a) {
    __shared__ unsigned long long s_cell[kLdsCells];
    __shared__ long long s_a0[kLdsCells];
    __shared__ long long s_a1[(AGG == GW_AVG_I64 || AGG == GW_AVG_F64) ? kLdsCells : 1];
    const int64_t tile = (int64_t)blockDim.x * kPreaggItems;
    const uint64_t R = (uint64_t)a.t.ring;
    const int64_t id0 = identity0(AGG);
    unsigned long long late = 0, ins = 0, flags = 0, occ = 0, cells = 0;
    for (int64_t t0 = blockIdx.x * tile; t0 < a.n; t0 += (int64_t)gridDim.x * tile) {
        for (int j = threadIdx.x; j < kLdsCells; j += blockDim.x) {
            s_cell[j] = ~0ull;
            s_a0[j] = id0;
            if constexpr (AGG == GW_AVG_I64 || AGG == GW_AVG_F64) s_a1[j] = 0;
        }
        __syncthreads();
#pragma unroll 1
        for (int it = 0; it < kPreaggItems; ++it) {
            const int64_t i = t0 + (int64_t)it * blockDim.x + threadIdx.x;
            bool defer = false;
            int64_t key = 0, pane = 0, c0 = 0, c1 = 0;
            if (i < a.n) {
                key = a.key[i];
                const int64_t ts = a.ts[i];
                const int64_t v = a.val ? a.val[i] : 0;
                if (ts == INT64_MIN) {
                    flags |= GW_DF_NO_TS;
                } else if (ts < a.t_late) {
                    if (a.late_exact) late++;
                    else flags |= GW_DF_RANGE;
                } else {
                    const uint64_t q = udiv64((uint64_t)ts - (uint64_t)a.t_late, a.div);
                    record_cell(AGG, v, c0, c1);
                    const uint64_t rel = q - a.delta;
                    if (q >= a.delta && rel < R) {
                        uint32_t pos = (uint32_t)a.b_pos + (uint32_t)rel;
                        if (pos >= R) pos -= (uint32_t)R;
                        bool inserted;
                        const int64_t si = find_or_insert(a.t, key, inserted);
                        ins += inserted;
                        if (si < 0) {
                            flags |= GW_DF_TABLE_FULL;
                            defer = true;
                            pane = a.p_late + (int64_t)q;
                        } else {
                            occ |= 1ull << pos;
                            const unsigned long long cell = (unsigned long long)(si * (int64_t)R + pos);
                            uint32_t h = (uint32_t)slot_hash((int64_t)cell) & (kLdsCells - 1);
                            bool done = false;
                            for (int p = 0; p < 32 && !done; ++p) {
                                unsigned long long cur = s_cell[h];
                                if (cur == ~0ull) cur = atomicCAS(&s_cell[h], ~0ull, cell);
                                if (cur == ~0ull || cur == cell) {
                                    if constexpr (AGG == GW_COUNT || AGG == GW_SUM_I64 || AGG == GW_SUM_I32) {
                                        atomicAdd((unsigned long long*)&s_a0[h], (unsigned long long)c0);
                                    } else if constexpr (AGG == GW_SUM_F64) {
                                        atomicAdd((double*)&s_a0[h], bits_to_f64(c0));
                                    } else if constexpr (AGG == GW_MIN_I64 || AGG == GW_MIN_F64) {
                                        atomicMin(&s_a0[h], (long long)c0);
                                    } else if constexpr (AGG == GW_MAX_I64 || AGG == GW_MAX_F64) {
                                        atomicMax(&s_a0[h], (long long)c0);
                                    } else if constexpr (AGG == GW_AVG_I64) {
                                        atomicAdd((unsigned long long*)&s_a0[h], (unsigned long long)c0);
                                        atomicAdd((unsigned long long*)&s_a1[h], (unsigned long long)c1);
                                    } else {
                                        atomicAdd((double*)&s_a0[h], bits_to_f64(c0));
                                        atomicAdd((unsigned long long*)&s_a1[h], (unsigned long long)c1);
                                    }
                                    done = true;
                                }
                                h = (h + 1) & (kLdsCells - 1);
                            }
                            if (!done) {  // LDS table saturated: straight to HBM
                                int64_t* s = slot_ptr(a.t, si);
                                cell_atomic<AGG>(s + 2 + pos * (uint32_t)a.t.words, c0, c1);
                                const unsigned long long bit = 1ull << pos;
                                if constexpr (uses_mask<AGG>()) {
                                    if (!(*(volatile unsigned long long*)(s + 1) & bit))
                                        atomicOr((unsigned long long*)(s + 1), bit);
                                }
                            }
                        }
                    } else {
                        if (q > (uint64_t)(INT64_MAX - a.p_late)) flags |= GW_DF_RANGE;
                        defer = true;
                        pane = a.p_late + (int64_t)q;
                    }
                }
            }
            const unsigned long long off = wave_reserve(&a.st->n_deferred, defer);
            if (defer) {
                a.d_key[off] = key;
                a.d_pane[off] = pane;
                a.d_a0[off] = c0;
                a.d_a1[off] = c1;
            }
        }
        __syncthreads();
        for (int j = threadIdx.x; j < kLdsCells; j += blockDim.x) {
            const unsigned long long cellu = s_cell[j];
            if (cellu == ~0ull) continue;
            const int64_t cell = (int64_t)cellu;
            cells++;
            const int64_t si = cell / (int64_t)R;
            const uint32_t pos = (uint32_t)(cell - si * (int64_t)R);
            int64_t* s = slot_ptr(a.t, si);
            int64_t b1 = 0;
            if constexpr (AGG == GW_AVG_I64 || AGG == GW_AVG_F64) b1 = s_a1[j];
            cell_atomic<AGG>(s + 2 + pos * (uint32_t)a.t.words, s_a0[j], b1);
            const unsigned long long bit = 1ull << pos;
            if constexpr (uses_mask<AGG>()) {
                if (!(*(volatile unsigned long long*)(s + 1) & bit)) atomicOr((unsigned long long*)(s + 1), bit);
            }
        }
        __syncthreads();
    }
    block_commit(a.st, late, ins, flags, occ, cells);
}

// Re-ingest parked partial aggregates whose pane now lies inside the ring.
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
                const int64_t si = find_or_insert(a.t, key, inserted);
                ins += inserted;
                if (si < 0) {
                    flags |= GW_DF_TABLE_FULL;
                    keep = true;
                } else {
                    int64_t* s = slot_ptr(a.t, si);
                    cell_atomic<AGG>(s + 2 + pos * a.t.words, c0, c1);
                    const unsigned long long bit = 1ull << pos;
                    if constexpr (uses_mask<AGG>()) {
                        if (!(*(volatile unsigned long long*)(s + 1) & bit))
                            atomicOr((unsigned long long*)(s + 1), bit);
                    }
                    occ |= bit;
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
// non-null pane among the nwin windows of this pass, then retires the panes that no
// later window covers (clearAllState).  Each block sweeps a contiguous chunk; rows
// are staged in LDS and flushed with one device atomic per 2048 rows (coalesced).
template <int AGG>
__global__ void __launch_bounds__(256) k_fire(FireArgs a) {
    __shared__ RowStage rs;
    const int64_t nslots = a.t.cap + 1;
    const int64_t id0 = identity0(AGG);
    const int W = a.t.words;
    const int R = a.t.ring;
    if (threadIdx.x == 0) rs.cnt = 0;
    if (blockIdx.x == 0 && threadIdx.x < kShards) atomicAnd(&a.st->sh[threadIdx.x].occ, ~a.rmask);
    __syncthreads();
    const int64_t chunk = ((nslots + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
    const int64_t c0 = blockIdx.x * chunk, c1 = min(nslots, c0 + chunk);
    for (int64_t base = c0; base < c1; base += blockDim.x) {
        const int64_t i = base + threadIdx.x;
        int64_t key = kEmptyKey;
        uint64_t mask = 0;
        int64_t* s = nullptr;
        if (i < c1) {
            s = slot_ptr(a.t, i);
            key = s[0];
            mask = presence<AGG>(s, R, W);
        }
        for (int w = 0; w < a.nwin; ++w) {
            // uniform flush decision: every thread reads rs.cnt before anyone appends
            const bool flush = rs.cnt + blockDim.x > kRowStage;
            __syncthreads();
            if (flush) stage_flush(rs, &a.st->rows, a.o_key, a.o_start, a.o_end, a.o_res);
            uint64_t m = mask & a.wmask[w];
            if (m) {
                int64_t r0 = id0, r1 = 0;
                while (m) {
                    const int pos = __ffsll((long long)m) - 1;
                    m &= m - 1;
                    const int64_t* c = s + 2 + pos * W;
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
        uint64_t m = mask & a.rmask;
        if (m) {
            if constexpr (uses_mask<AGG>()) s[1] = (int64_t)(mask & ~a.rmask);
            while (m) {
                const int pos = __ffsll((long long)m) - 1;
                m &= m - 1;
                s[2 + pos * W] = id0;
                if (W == 2) s[3 + pos * W] = 0;
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
        const int64_t i = base + threadIdx.x;
        uint64_t m = 0;
        int64_t* s = nullptr;
        int64_t key = 0;
        if (i < nslots) {
            s = slot_ptr(a.t, i);
            key = s[0];
            m = presence<AGG>(s, a.t.ring, W) & a.emask;
        }
        unsigned long long off = wave_reserve_n(&a.st->n_deferred, (unsigned)__popcll(m));
        if (m) {
            if constexpr (uses_mask<AGG>()) s[1] = (int64_t)((uint64_t)s[1] & ~a.emask);
            while (m) {
                const int pos = __ffsll((long long)m) - 1;
                m &= m - 1;
                int64_t* c = s + 2 + pos * W;
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

// Re-hash live slots (mask != 0) into a fresh table; dead keys are dropped.
__global__ void __launch_bounds__(256) k_rehash(TableView o, TableView n, DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    const int64_t nslots = o.cap + 1;
    const int W = o.stride_w;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nslots;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t* s = slot_ptr(o, i);
        if (presence_rt(s, o) == 0) continue;
        const int64_t key = i == o.cap ? kEmptyKey : s[0];
        bool inserted;
        const int64_t j = find_or_insert(n, key, inserted);
        if (j < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        ins += inserted;
        int64_t* d = slot_ptr(n, j);
        for (int w = 1; w < W; ++w) d[w] = s[w];
    }
    block_commit(st, 0, ins, flags, 0);
}

__global__ void __launch_bounds__(256) k_count_live(TableView t, unsigned long long* out) {
    unsigned long long c = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= t.cap;
         i += (int64_t)gridDim.x * blockDim.x)
        c += presence_rt(slot_ptr(t, i), t) != 0;
    wave_add(out, c);
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

hipError_t launch_table_init(const TableView& t, hipStream_t s) {
#define L(A) hipLaunchKernelGGL(k_table_init<A>, dim3(grid_for(t.cap + 1)), dim3(256), 0, s, t)
    GW_AGG_SWITCH(t.agg, L);
#undef L
    return hipGetLastError();
}

hipError_t launch_ingest(const IngestArgs& a, bool preagg, int unroll, hipStream_t s) {
    if (preagg) {
        const int g = grid_for(a.n, kPreaggItems);
#define L(A) hipLaunchKernelGGL(k_ingest_preagg<A>, dim3(g), dim3(256), 0, s, a)
        GW_AGG_SWITCH(a.t.agg, L);
#undef L
    } else {
        if (unroll == 4) {
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

hipError_t launch_count_live(const TableView& t, unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(k_count_live, dim3(grid_for(t.cap + 1)), dim3(256), 0, s, t, out);
    return hipGetLastError();
}

hipError_t launch_rehash(const TableView& o, const TableView& n, DevStatus* st, hipStream_t s) {
    hipLaunchKernelGGL(k_rehash, dim3(grid_for(o.cap + 1)), dim3(256), 0, s, o, n, st);
    return hipGetLastError();
}

}  // namespace gw
