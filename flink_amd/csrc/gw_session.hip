// gw_session.hip — event-time session windows (gap merge) on gfx950.
//
// Reference semantics (paths relative to the Flink tree):
//   EventTimeSessionWindows.assignWindows -> [ts, ts + gap)
//     (flink-streaming-java/.../api/windowing/assigners/EventTimeSessionWindows.java:61-64)
//   TimeWindow.intersects (inclusive: touching windows merge) / cover / mergeWindows
//     (RS/api/windowing/windows/TimeWindow.java:116-123,208-254)
//   MergingWindowSet.addWindow (RS/runtime/operators/windowing/MergingWindowSet.java:153-224)
//   WindowOperator.processElement merging branch incl. "drop if the window is already
//     late" (RS/runtime/operators/windowing/WindowOperator.java:303-403)
//   AbstractHeapMergingState.mergeNamespaces (RR/state/heap/AbstractHeapMergingState.java:65-91)
//   EventTimeTrigger + onEventTime: a session fires once when end-1 <= watermark.
//
// MI355X design: per watermark batch, records are grouped by (state
// slot, timestamp) with a hand-written radix sort; each slot's sorted records are
// swept against its in-flight sessions (<= K kept inline in the 64/128-byte slot).
// Without late records the result of the reference's record-at-a-time merging is the
// set of connected components of all windows (inclusive intersection), which a
// sorted sweep computes in one pass.  If a slot's batch holds a record whose own
// window is already late, the reference's outcome depends on arrival order (a late
// window is dropped unless it touches an in-flight session at that moment), so that
// slot is replayed record by record in arrival order.
#include "gw_kernels.h"
#include "gw_session.h"
#include "gw_sort.h"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <vector>

namespace gw {

constexpr int kMaxLocalSess = 32;

struct SegArgs {
    const uint64_t* skey;   // sorted (slot << ts_bits) | (ts - ts_min)
    const uint32_t* perm;   // original record index
    int64_t n;
    int ts_bits;
    int64_t ts_min;
    const int64_t* val;
    int64_t gap;
    int64_t wm;             // current watermark (all records of the batch see it)
    int64_t lateness;       // allowed lateness (WindowOperator.allowedLateness)
    int purge;              // PurgingTrigger with lateness > 0: a fired session keeps an empty state
    int64_t* o_key;         // rows of windows an element fires at once (EventTimeTrigger.onElement
    int64_t* o_start;       //   FIRE: window max timestamp <= watermark; lateness > 0 only)
    int64_t* o_end;
    int64_t* o_res;
    TableView t;            // ring = K sessions per slot, words = words per session
    const int64_t* ts;      // the batch's columns (late side output)
    const int64_t* key;
    int64_t* lo_key;        // late side output (GW_FLAG_LATE_SIDE_OUTPUT), append at st->n_late_out;
    int64_t* lo_ts;         //   nullptr: late elements are counted (numLateRecordsDropped)
    int64_t* lo_val;
    const uint32_t* retry_in;
    int64_t n_retry_in;
    uint32_t* retry_out;    // appended at st->overflow
    DevStatus* st;
};

__global__ void __launch_bounds__(256) k_sess_minmax(const int64_t* ts, int64_t n, long long* mm,
                                                     DevStatus* st) {
    long long lo = INT64_MAX, hi = INT64_MIN;
    unsigned long long flags = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const long long t = ts[i];
        if (t == INT64_MIN) { flags |= GW_DF_NO_TS; continue; }
        lo = t < lo ? t : lo;
        hi = t > hi ? t : hi;
    }
    for (int o = 32; o > 0; o >>= 1) {
        long long a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    __shared__ long long red[2][16];
    const int wave = threadIdx.x >> 6;
    if (__lane_id() == 0) { red[0][wave] = lo; red[1][wave] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
            lo = red[0][w] < lo ? red[0][w] : lo;
            hi = red[1][w] > hi ? red[1][w] : hi;
        }
        if (lo != INT64_MAX) atomicMin(&mm[0], lo);
        if (hi != INT64_MIN) atomicMax(&mm[1], hi);
    }
    block_commit(st, 0, 0, flags, 0);
}

__global__ void __launch_bounds__(256) k_sess_prep(const int64_t* key, const int64_t* ts, int64_t n, int64_t ts_min,
                                                   int ts_bits, TableView t, uint64_t* skey, uint32_t* perm,
                                                   DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool inserted;
        int64_t s = find_or_insert(t, key[i], inserted);
        ins += inserted;
        if (s < 0) { flags |= GW_DF_TABLE_FULL; s = 0; }
        skey[i] = ((uint64_t)s << ts_bits) | (uint64_t)(ts[i] - ts_min);
        perm[i] = (uint32_t)i;
    }
    block_commit(st, 0, ins, flags, 0);
}

struct Sess {
    int64_t s, e, a0, a1;
    bool f;  // its event-time timer has fired (kept for allowed lateness until cleanup)
};

// Slot word 1: in-flight session count (low 32 bits) | fired bit per session (high 32).
__device__ __forceinline__ int slot_cnt(int64_t w) { return (int)(uint32_t)(uint64_t)w; }
__device__ __forceinline__ bool slot_fired(int64_t w, int q) { return ((uint64_t)w >> (32 + q)) & 1ull; }

// WindowOperator.cleanupTime (:670-677, overflow -> Long.MAX_VALUE, never cleaned) <= wm
__device__ __forceinline__ bool cleaned_at(int64_t end, int64_t lateness, int64_t wm) {
    const int64_t mx = end - 1;
    int64_t ct;
    if (__builtin_add_overflow(mx, lateness, &ct)) ct = INT64_MAX;
    return ct <= wm;
}

// The empty state a purged session keeps (FIRE_AND_PURGE clears the contents, the window
// stays in the merging window set until its cleanup time): the fold identity, with -0.0
// for floating sums so that folding a single -0.0 keeps its sign.
template <int AGG>
__device__ __forceinline__ void purge_acc(int64_t& a0, int64_t& a1) {
    a0 = AGG == GW_AVG_F64 ? (int64_t)0x8000000000000000ull : identity0(AGG);
    a1 = 0;
}

template <int AGG>
__device__ __forceinline__ void emit_now(const SegArgs& a, int64_t key, const Sess& x) {
    const unsigned long long at = atomicAdd(&a.st->rows, 1ull);
    a.o_key[at] = key;
    a.o_start[at] = x.s;
    a.o_end[at] = x.e;
    a.o_res[at] = cell_result(AGG, x.a0, x.a1);
}

template <int AGG>
__device__ void seg_process(const SegArgs& a, int64_t i) {
    const uint64_t tsmask = (a.ts_bits >= 64) ? ~0ull : ((1ull << a.ts_bits) - 1ull);
    const int64_t slot = (int64_t)(a.skey[i] >> a.ts_bits);
    int64_t j = i + 1;
    while (j < a.n && (int64_t)(a.skey[j] >> a.ts_bits) == slot) ++j;
    int64_t* sp = slot_ptr(a.t, slot);
    const int SW = a.t.words;
    const int K = a.t.ring;
    Sess cur_list[kMaxLocalSess];
    const int64_t w1 = sp[1];
    int cnt = slot_cnt(w1);
    for (int q = 0; q < cnt; ++q) {
        const int64_t* x = sp + 2 + q * SW;
        cur_list[q] = Sess{x[0], x[1], x[2], SW == 4 ? x[3] : 0, slot_fired(w1, q)};
    }
    unsigned long long late = 0, merges = 0, flags = 0;
    const int64_t ts_first = a.ts_min + (int64_t)(a.skey[i] & tsmask);
    bool ok = true;
    if ((uint64_t)ts_first > (uint64_t)INT64_MAX - (uint64_t)a.gap && ts_first > 0) flags |= GW_DF_RANGE;
    const bool any_late = ts_first + a.gap - 1 <= a.wm;  // sorted by ts: the first is the earliest
    if (!any_late) {
        // Sweep old sessions and the batch's windows in start order; merge on inclusive intersect.
        Sess out[kMaxLocalSess];
        int nout = 0, oi = 0;
        int64_t e = i;
        bool have = false;
        bool cur_has_state = false;
        Sess cur{0, 0, 0, 0};
        while (oi < cnt || e < j) {
            Sess item;
            bool is_old;
            const int64_t te = e < j ? a.ts_min + (int64_t)(a.skey[e] & tsmask) : INT64_MAX;
            if (oi < cnt && (e >= j || cur_list[oi].s <= te)) {
                item = cur_list[oi++];
                is_old = true;
            } else {
                int64_t c0, c1;
                record_cell(AGG, a.val ? a.val[a.perm[e]] : 0, c0, c1);
                item = Sess{te, te + a.gap, c0, c1, false};
                is_old = false;
                ++e;
            }
            if (!have) {
                cur = item;
                have = true;
                cur_has_state = is_old;
            } else if (item.s <= cur.e) {
                if (item.e > cur.e) cur.e = item.e;
                fold_cell(AGG, cur.a0, cur.a1, item.a0, item.a1);
                cur.f = cur.f && item.f;  // a merge with a new window re-arms the timer (its end > wm)
                if (is_old && cur_has_state) merges++;
                cur_has_state |= is_old;
            } else {
                if (nout == kMaxLocalSess) { ok = false; break; }
                out[nout++] = cur;
                cur = item;
                cur_has_state = is_old;
            }
        }
        if (ok && have) {
            if (nout == kMaxLocalSess) ok = false;
            else out[nout++] = cur;
        }
        if (ok) {
            for (int q = 0; q < nout; ++q) cur_list[q] = out[q];
            cnt = nout;
        }
    } else {
        // Arrival-order replay (MergingWindowSet.addWindow per record).  With allowed
        // lateness an element may fire its window at once; those rows are written only in
        // a second pass, once the first has shown that the result fits the slot (a slot
        // that overflows is retried after widening and must not emit twice).
        Sess init[kMaxLocalSess];
        const int cnt0 = cnt;
        const int passes = (a.lateness > 0 || a.lo_key) ? 2 : 1;
        for (int q = 0; q < cnt0 && passes == 2; ++q) init[q] = cur_list[q];
        for (int pass = 0; pass < passes; ++pass) {
        const bool emit = pass == 1;
        if (emit) {
            if (!ok || cnt > K) break;
            for (int q = 0; q < cnt0; ++q) cur_list[q] = init[q];
            cnt = cnt0;
            late = 0;
            merges = 0;
        }
        int64_t last = -1;
        for (int64_t step = i; step < j && ok; ++step) {
            int64_t best = -1;
            uint32_t bp = 0xffffffffu;
            for (int64_t x = i; x < j; ++x) {
                const uint32_t p = a.perm[x];
                if ((int64_t)p > last && p < bp) { bp = p; best = x; }
            }
            last = bp;
            const int64_t ts = a.ts_min + (int64_t)(a.skey[best] & tsmask);
            const int64_t ws = ts, we = ts + a.gap;
            int lo = -1, hi = -1;
            for (int q = 0; q < cnt; ++q) {
                if (cur_list[q].s <= we && cur_list[q].e >= ws) {
                    if (lo < 0) lo = q;
                    hi = q;
                }
            }
            int64_t c0, c1;
            record_cell(AGG, a.val ? a.val[bp] : 0, c0, c1);
            if (lo < 0) {
                if (cleaned_at(we, a.lateness, a.wm)) {  // isWindowLate: skipped, and the element is late
                    if (!a.lo_key) { late++; continue; }
                    if (emit) {  // sideOutput(element) (WindowOperator.java:440-446, 587-588)
                        const unsigned long long o = atomicAdd(&a.st->n_late_out, 1ull);
                        a.lo_key[o] = a.key[bp];
                        a.lo_ts[o] = a.ts[bp];
                        a.lo_val[o] = a.val ? a.val[bp] : 0;
                    }
                    continue;
                }
                if (cnt == kMaxLocalSess) { ok = false; break; }
                int q = cnt;
                while (q > 0 && cur_list[q - 1].s > ws) { cur_list[q] = cur_list[q - 1]; --q; }
                cur_list[q] = Sess{ws, we, c0, c1, we - 1 <= a.wm};
                if (cur_list[q].f) {  // onElement: FIRE (PurgingTrigger: FIRE_AND_PURGE)
                    if (emit) emit_now<AGG>(a, sp[0], cur_list[q]);
                    if (a.purge) purge_acc<AGG>(cur_list[q].a0, cur_list[q].a1);
                }
                cnt++;
            } else {
                Sess m = cur_list[lo];
                if (ws < m.s) m.s = ws;
                for (int q = lo + 1; q <= hi; ++q) {
                    if (cur_list[q].e > m.e) m.e = cur_list[q].e;
                    fold_cell(AGG, m.a0, m.a1, cur_list[q].a0, cur_list[q].a1);
                    merges++;
                }
                if (we > m.e) m.e = we;
                fold_cell(AGG, m.a0, m.a1, c0, c1);
                m.f = m.e - 1 <= a.wm;  // onElement FIRE, or onMerge registers the merged window's timer
                if (m.f) {
                    if (emit) emit_now<AGG>(a, sp[0], m);
                    if (a.purge) purge_acc<AGG>(m.a0, m.a1);
                }
                cur_list[lo] = m;
                const int removed = hi - lo;
                for (int q = hi + 1; q < cnt; ++q) cur_list[q - removed] = cur_list[q];
                cnt -= removed;
            }
        }
        }
    }
    if (!ok || cnt > K) {
        // does not fit the slot: leave the slot untouched, retry after widening
        const unsigned long long at = atomicAdd(&a.st->overflow, 1ull);
        a.retry_out[at] = (uint32_t)i;
        atomicMax(&a.st->pad[1], (unsigned long long)(ok ? cnt : kMaxLocalSess + 1));
        return;
    }
    uint64_t fired = 0;
    for (int q = 0; q < cnt; ++q) {
        int64_t* x = sp + 2 + q * SW;
        x[0] = cur_list[q].s;
        x[1] = cur_list[q].e;
        x[2] = cur_list[q].a0;
        if (SW == 4) x[3] = cur_list[q].a1;
        fired |= (uint64_t)cur_list[q].f << q;
    }
    sp[1] = (int64_t)(((uint64_t)fired << 32) | (uint64_t)(uint32_t)cnt);
    ShardCtr& sc = a.st->sh[blockIdx.x % kShards];
    if (late) atomicAdd(&sc.late, late);
    if (merges) atomicAdd(&sc.merges, merges);
    if (flags) atomicOr(&sc.flags, flags);
}

template <int AGG>
__global__ void __launch_bounds__(256) k_sess_segment(SegArgs a) {
    if (a.retry_in) {
        for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < a.n_retry_in;
             r += (int64_t)gridDim.x * blockDim.x)
            seg_process<AGG>(a, (int64_t)a.retry_in[r]);
        return;
    }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i > 0 && (a.skey[i] >> a.ts_bits) == (a.skey[i - 1] >> a.ts_bits)) continue;
        seg_process<AGG>(a, i);
    }
}

// Fire every in-flight session with end-1 <= wm (sessions in a slot are disjoint and
// sorted, so the fired ones are a prefix), emit (key, start, end, result), purge.
// Rows are staged in LDS, one row per thread per round, and flushed in bulk.
template <int AGG>
__global__ void __launch_bounds__(256) k_sess_fire(TableView t, int64_t wm, int64_t lateness, int purge, int64_t* o_key,
                                                   int64_t* o_start, int64_t* o_end, int64_t* o_res, DevStatus* st) {
    __shared__ RowStage rs;
    __shared__ int s_max;
    const int64_t nslots = t.cap + 1;
    const int SW = t.words;
    if (threadIdx.x == 0) rs.cnt = 0;
    __syncthreads();
    const int64_t chunk = ((nslots + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
    const int64_t c0 = blockIdx.x * chunk, c1 = min(nslots, c0 + chunk);
    for (int64_t base = c0; base < c1; base += blockDim.x) {
        const int64_t i = base + threadIdx.x;
        int64_t* s = nullptr;
        int cnt = 0, nf = 0, nc = 0;
        int64_t w1 = 0;
        if (i < c1) {
            s = slot_ptr(t, i);
            w1 = s[1];
            cnt = slot_cnt(w1);
            while (nf < cnt && s[2 + nf * SW + 1] - 1 <= wm) ++nf;  // due timers: a prefix (sorted, disjoint)
            nc = nf;
            if (lateness > 0) {  // cleanup timers (max timestamp + lateness) are a prefix of those
                nc = 0;
                while (nc < nf && cleaned_at(s[2 + nc * SW + 1], lateness, wm)) ++nc;
            }
        }
        if (threadIdx.x == 0) s_max = 0;
        __syncthreads();
        if (nf) atomicMax(&s_max, nf);
        __syncthreads();
        const int rounds = s_max;
        __syncthreads();  // everyone has read s_max before thread 0 resets it
        for (int q = 0; q < rounds; ++q) {
            const bool flush = rs.cnt + blockDim.x > kRowStage;
            __syncthreads();
            if (flush) stage_flush(rs, &st->rows, o_key, o_start, o_end, o_res);
            if (q < nf && !slot_fired(w1, q)) {
                const int64_t* x = s + 2 + q * SW;
                const unsigned j = atomicAdd(&rs.cnt, 1u);
                rs.k[j] = s[0];
                rs.s[j] = x[0];
                rs.e[j] = x[1];
                rs.r[j] = cell_result(AGG, x[2], SW == 4 ? x[3] : 0);
            }
            __syncthreads();
        }
        if (nf) {
            uint64_t fired = 0;
            for (int q = nc; q < cnt; ++q) {
                for (int w = 0; w < SW; ++w) s[2 + (q - nc) * SW + w] = s[2 + q * SW + w];
                fired |= (uint64_t)(q < nf || slot_fired(w1, q)) << (q - nc);
                if (purge && q < nf && !slot_fired(w1, q)) {  // FIRE_AND_PURGE of a kept session
                    int64_t z0, z1;
                    purge_acc<AGG>(z0, z1);
                    s[2 + (q - nc) * SW + 2] = z0;
                    if (SW == 4) s[2 + (q - nc) * SW + 3] = z1;
                }
            }
            s[1] = (int64_t)((fired << 32) | (uint64_t)(uint32_t)(cnt - nc));
        }
    }
    stage_flush(rs, &st->rows, o_key, o_start, o_end, o_res);
}

__global__ void __launch_bounds__(256) k_sess_rewiden(TableView o, TableView n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= o.cap; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t* s = slot_ptr(o, i);
        int64_t* d = slot_ptr(n, i);
        d[0] = s[0];
        d[1] = s[1];
        const int cnt = slot_cnt(s[1]);
        for (int w = 0; w < cnt * o.words; ++w) d[2 + w] = s[2 + w];
    }
}

// Re-hash slots with in-flight sessions into a fresh table (dead keys dropped).
__global__ void __launch_bounds__(256) k_sess_rehash(TableView o, TableView n, DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= o.cap; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t* s = slot_ptr(o, i);
        if (s[1] == 0) continue;
        const int64_t key = i == o.cap ? kEmptyKey : s[0];
        bool inserted;
        const int64_t j = find_or_insert(n, key, inserted);
        if (j < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        ins += inserted;
        int64_t* d = slot_ptr(n, j);
        const int cnt = slot_cnt(s[1]);
        d[1] = s[1];
        for (int w = 0; w < cnt * o.words; ++w) d[2 + w] = s[2 + w];
    }
    block_commit(st, 0, ins, flags, 0);
}

__global__ void __launch_bounds__(256) k_sess_init(TableView t) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= t.cap; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t* s = slot_ptr(t, i);
        s[0] = kEmptyKey;
        s[1] = 0;
    }
}

// Restore (gw_restore of a session snapshot): one thread per restored key.  The key's
// restored sessions (sorted by start, disjoint) are swept together with the slot's
// in-flight ones in start order and merged on inclusive intersection, exactly as
// seg_process merges a batch; a fresh slot receives them unchanged.  A key whose
// result exceeds the slot's K sessions is counted in st->overflow and left untouched.
template <int AGG>
__global__ void __launch_bounds__(256) k_sess_restore(TableView t, const int64_t* rk, const int64_t* roff,
                                                      const int64_t* rs, int64_t n, DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool inserted;
        const int64_t slot = find_or_insert(t, rk[i], inserted);
        ins += inserted;
        if (slot < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        int64_t* sp = slot_ptr(t, slot);
        const int SW = t.words, K = t.ring;
        const int64_t w1 = sp[1];
        const int cnt = slot_cnt(w1);
        Sess out[kMaxLocalSess];
        int nout = 0, oi = 0;
        int64_t r = roff[i];
        const int64_t re = roff[i + 1];
        bool have = false, ok = true;
        Sess cur{0, 0, 0, 0};
        while (oi < cnt || r < re) {
            Sess item;
            const int64_t* x = sp + 2 + oi * SW;
            if (oi < cnt && (r >= re || x[0] <= rs[r * 5])) {
                item = Sess{x[0], x[1], x[2], SW == 4 ? x[3] : 0, slot_fired(w1, oi)};
                ++oi;
            } else {
                item = Sess{rs[r * 5], rs[r * 5 + 1], rs[r * 5 + 2], rs[r * 5 + 3], rs[r * 5 + 4] != 0};
                ++r;
            }
            if (!have) {
                cur = item;
                have = true;
            } else if (item.s <= cur.e) {
                if (item.e > cur.e) cur.e = item.e;
                fold_cell(AGG, cur.a0, cur.a1, item.a0, item.a1);
                cur.f = cur.f && item.f;
            } else {
                if (nout == K) { ok = false; break; }
                out[nout++] = cur;
                cur = item;
            }
        }
        if (ok && have) {
            if (nout == K) ok = false;
            else out[nout++] = cur;
        }
        if (!ok) {
            atomicAdd(&st->overflow, 1ull);
            continue;
        }
        uint64_t fired = 0;
        for (int q = 0; q < nout; ++q) {
            int64_t* y = sp + 2 + q * SW;
            y[0] = out[q].s;
            y[1] = out[q].e;
            y[2] = out[q].a0;
            if (SW == 4) y[3] = out[q].a1;
            fired |= (uint64_t)out[q].f << q;
        }
        sp[1] = (int64_t)((fired << 32) | (uint64_t)(uint32_t)nout);
    }
    block_commit(st, 0, ins, flags, 0);
}

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

static unsigned grid_of(int64_t n) {
    int64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    return (unsigned)g;
}

// --------------------------------------------------------------------------- count windows
// KeyedStream.countWindow(size) / countWindow(size, slide) over GlobalWindows
// (RS/api/datastream/KeyedStream.java:676-690): CountTrigger fires on the element that
// brings the key's count to a multiple of the trigger count (CountTrigger.java:47-56);
// the tumbling form purges (PurgingTrigger.onElement :44-48), the sliding form evicts
// all but the newest `size` elements before the function (CountEvictor.java:50-85).
//
// MI355X design: the elements of a key are cut into count-panes of g = gcd(size, slide)
// consecutive elements, so every fired window is exactly n = size/g whole panes (the
// first windows of a key: all its panes so far) and every slide ends a pane.  A slot
// holds [key][element count][ring of n pane accumulators]; a batch is grouped by slot
// with the stable radix sort (arrival order kept inside a key) and each key's run is
// folded in order by one thread, which emits a row at every multiple of the slide.
struct CountGeom {
    int64_t size, slide, g;
};

__global__ void __launch_bounds__(256) k_cnt_slot(TableView t, const int64_t* key, int64_t n, uint64_t* kslot,
                                                  uint32_t* idx, DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool inserted;
        const int64_t j = find_or_insert(t, key[i], inserted);
        if (j < 0) flags |= GW_DF_TABLE_FULL;
        ins += inserted;
        kslot[i] = j < 0 ? (uint64_t)t.cap + 1 : (uint64_t)j;  // cap + 1: parked, never applied
        idx[i] = (uint32_t)i;
    }
    block_commit(st, 0, ins, flags, 0);
}

template <int AGG>
__global__ void __launch_bounds__(256) k_cnt_apply(TableView t, CountGeom G, const uint64_t* ks, const uint32_t* perm,
                                                   int64_t n, const int64_t* val, int64_t* ok, int64_t* os,
                                                   int64_t* oe, int64_t* orr, DevStatus* st) {
    constexpr int W = (AGG == GW_AVG_I64 || AGG == GW_AVG_F64) ? 2 : 1;
    const int R = t.ring;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t slot = ks[i];
        if ((i > 0 && ks[i - 1] == slot) || slot > (uint64_t)t.cap) continue;  // not the head of a key's run
        int64_t* sp = slot_ptr(t, (int64_t)slot);
        int64_t* cells = sp + 2;
        const int64_t key = sp[0];  // the sentinel slot's key word is Long.MIN_VALUE, its key
        int64_t c = sp[1];
        for (int64_t r = i; r < n && ks[r] == slot; ++r) {
            int64_t a0, a1;
            record_cell(AGG, val ? val[perm[r]] : 0, a0, a1);
            int64_t* cell = cells + ((c / G.g) % R) * W;
            if (c % G.g == 0) {  // first element of a pane: the ring cell starts over
                cell[0] = a0;
                if (W == 2) cell[1] = a1;
            } else {
                int64_t b0 = cell[0], b1 = W == 2 ? cell[1] : 0;
                fold_cell(AGG, b0, b1, a0, a1);
                cell[0] = b0;
                if (W == 2) cell[1] = b1;
            }
            ++c;
            if (c % G.slide == 0) {  // CountTrigger FIRE: the newest min(size, c) elements
                const int64_t len = c < G.size ? c : G.size;
                const int64_t p0 = (c - len) / G.g, p1 = c / G.g;
                const int64_t* f = cells + (p0 % R) * W;
                int64_t r0 = f[0], r1 = W == 2 ? f[1] : 0;
                for (int64_t q = p0 + 1; q < p1; ++q) {
                    const int64_t* e = cells + (q % R) * W;
                    fold_cell(AGG, r0, r1, e[0], W == 2 ? e[1] : 0);
                }
                const unsigned long long o = atomicAdd(&st->rows, 1ull);
                ok[o] = key;
                os[o] = c - len;
                oe[o] = c;
                orr[o] = cell_result(AGG, r0, r1);
            }
        }
        sp[1] = c;
    }
}

__global__ void __launch_bounds__(256) k_cnt_rehash(TableView o, TableView nt, DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    const int words = o.ring * o.words;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= o.cap; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t* sp = slot_ptr(o, i);
        if (sp[1] == 0) continue;  // every key in the table has counted an element
        const int64_t key = i == o.cap ? kEmptyKey : sp[0];
        bool inserted;
        const int64_t j = find_or_insert(nt, key, inserted);
        if (j < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        ins += inserted;
        int64_t* d = slot_ptr(nt, j);
        d[1] = sp[1];
        for (int w = 0; w < words; ++w) d[2 + w] = sp[2 + w];
    }
    block_commit(st, 0, ins, flags, 0);
}

// Restore of count-window state: one thread per entry (key, element count, ring of pane
// accumulators), copied into the key's slot.  The slot geometry is a function of the
// configuration (checked by the caller), so the copy is exact.  A key that already holds
// state here is counted in st->overflow and left untouched (blobs of one key group are
// never restored twice).
__global__ void __launch_bounds__(256) k_cnt_restore(TableView t, const int64_t* ent, int64_t n, DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    const int words = t.ring * t.words;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t* e = ent + i * (2 + words);
        bool inserted;
        const int64_t j = find_or_insert(t, e[0], inserted);
        if (j < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        ins += inserted;
        int64_t* d = slot_ptr(t, j);
        if (d[1] != 0) {
            atomicAdd(&st->overflow, 1ull);
            continue;
        }
        for (int w = 0; w < words; ++w) d[2 + w] = e[2 + w];
        d[1] = e[1];
    }
    block_commit(st, 0, ins, flags, 0);
}

// --------------------------------------------------------------------------- host
struct SessionState {
    gw_config cfg{};
    hipStream_t stream = nullptr;
    TableView tv{};
    DevStatus* d_st = nullptr;
    DevStatus* h_st = nullptr;
    long long* d_mm = nullptr;
    uint64_t* k0 = nullptr;
    uint64_t* k1 = nullptr;
    uint32_t* v0 = nullptr;
    uint32_t* v1 = nullptr;
    uint32_t* r0 = nullptr;
    uint32_t* r1 = nullptr;
    void* scratch = nullptr;
    int64_t buf_cap = 0;
    int64_t* o_key = nullptr;
    int64_t* o_start = nullptr;
    int64_t* o_end = nullptr;
    int64_t* o_res = nullptr;
    int64_t o_cap = 0;
    int64_t wm = INT64_MIN;
    gw_stats stats{};
    bool timing = false;
    bool count_mode = false;  // GW_COUNT_TUMBLING / GW_COUNT_SLIDING (same slot table and row plumbing)
    CountGeom cg{};
    int64_t* lo_buf[3] = {nullptr, nullptr, nullptr};  // late side output: key | ts | value
    int64_t lo_cap = 0, lo_head = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending[2], ev_pool;
    double t_total[2] = {0, 0};
    int64_t t_count[2] = {0, 0};
};

static int dev_err(std::string& err, const char* what, hipError_t e) {
    char b[256];
    snprintf(b, sizeof(b), "%s: %s", what, hipGetErrorString(e));
    err = b;
    return GW_E_DEVICE;
}
#define SCHECK(x)                                        \
    do {                                                 \
        hipError_t e_ = (x);                             \
        if (e_ != hipSuccess) return dev_err(err, #x, e_); \
    } while (0)

static void resolve_timers(SessionState* s) {
    for (int w = 0; w < 2; ++w) {
        for (auto& p : s->ev_pending[w]) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) { s->t_total[w] += ms; s->t_count[w]++; }
            s->ev_pool.push_back(p);
        }
        s->ev_pending[w].clear();
    }
}
static std::pair<hipEvent_t, hipEvent_t> get_ev(SessionState* s) {
    if (!s->ev_pool.empty()) { auto p = s->ev_pool.back(); s->ev_pool.pop_back(); return p; }
    std::pair<hipEvent_t, hipEvent_t> p;
    hipEventCreate(&p.first);
    hipEventCreate(&p.second);
    return p;
}

int session_refresh(SessionState* s, std::string& err) {
    SCHECK(hipMemcpyAsync(s->h_st, s->d_st, sizeof(DevStatus), hipMemcpyDeviceToHost, s->stream));
    SCHECK(hipStreamSynchronize(s->stream));
    fold_shards(s->h_st);
    if (s->timing) resolve_timers(s);
    if (s->h_st->flags & GW_DF_NO_TS) {
        err = "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Did you forget to call "
              "'DataStream.assignTimestampsAndWatermarks(...)'?";
        return GW_E_NO_TIMESTAMP;
    }
    if (s->h_st->flags & GW_DF_RANGE) {
        err = "session window end overflows int64";
        return GW_E_RANGE;
    }
    return GW_OK;
}

static int set_word(SessionState* s, size_t off, unsigned long long v, std::string& err) {
    unsigned long long* hv = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(s->h_st) + off);
    *hv = v;
    SCHECK(hipMemcpyAsync(reinterpret_cast<char*>(s->d_st) + off, hv, 8, hipMemcpyHostToDevice, s->stream));
    SCHECK(hipStreamSynchronize(s->stream));
    return GW_OK;
}

static int alloc_sess_table(SessionState* s, TableView& t, int64_t cap, int K, std::string& err) {
    t = s->tv;
    t.cap = cap;
    t.ring = K;
    t.stride_w = (int)(((2 + K * t.words) + 7) / 8 * 8);
    SCHECK(hipMalloc((void**)&t.base, (size_t)(cap + 1) * t.stride_w * 8));
    hipLaunchKernelGGL(k_sess_init, dim3(grid_of(cap + 1)), dim3(256), 0, s->stream, t);
    SCHECK(hipGetLastError());
    return GW_OK;
}

int session_create(SessionState*& out, const gw_config& cfg, int64_t cap, hipStream_t stream, DevStatus*,
                   std::string& why) {
    SessionState* s = new SessionState();
    s->cfg = cfg;
    s->stream = stream;
    s->tv.agg = cfg.agg;
    s->tv.words = cell_words(cfg.agg) == 2 ? 4 : 3;
    std::string& err = why;
    SCHECK(hipMalloc((void**)&s->d_st, sizeof(DevStatus)));
    SCHECK(hipHostMalloc((void**)&s->h_st, sizeof(DevStatus), hipHostMallocDefault));
    SCHECK(hipMalloc((void**)&s->d_mm, 16));
    SCHECK(hipMemset(s->d_st, 0, sizeof(DevStatus)));
    memset(s->h_st, 0, sizeof(DevStatus));
    int rc;
    if (cfg.assigner == GW_COUNT_TUMBLING || cfg.assigner == GW_COUNT_SLIDING) {
        s->count_mode = true;
        const int64_t size = cfg.size, slide = cfg.assigner == GW_COUNT_SLIDING ? cfg.slide : cfg.size;
        int64_t a = size, b = slide;
        while (b) { const int64_t t = a % b; a = b; b = t; }
        s->cg = CountGeom{size, slide, a};
        s->tv.words = cell_words(cfg.agg);
        rc = alloc_sess_table(s, s->tv, cap, (int)(size / a), why);  // ring of size/g panes
        if (rc) { session_destroy(s); return rc; }
        out = s;
        return GW_OK;
    }
    // K so that the slot fills a 64-byte (sum/count/min/max) or 128-byte (avg) line
    const int K = s->tv.words == 3 ? 2 : 3;
    rc = alloc_sess_table(s, s->tv, cap, K, why);
    if (rc) { session_destroy(s); return rc; }
    out = s;
    return GW_OK;
}

void session_destroy(SessionState* s) {
    if (!s) return;
    hipStreamSynchronize(s->stream);
    hipFree(s->tv.base);
    hipFree(s->d_st);
    hipHostFree(s->h_st);
    hipFree(s->d_mm);
    hipFree(s->k0); hipFree(s->k1); hipFree(s->v0); hipFree(s->v1); hipFree(s->r0); hipFree(s->r1);
    hipFree(s->scratch);
    hipFree(s->o_key); hipFree(s->o_start); hipFree(s->o_end); hipFree(s->o_res);
    for (auto* p : s->lo_buf) hipFree(p);
    for (int w = 0; w < 2; ++w) for (auto& p : s->ev_pending[w]) s->ev_pool.push_back(p);
    for (auto& p : s->ev_pool) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    delete s;
}

static int ensure_bufs(SessionState* s, int64_t n, std::string& err) {
    if (n <= s->buf_cap) return GW_OK;
    const int64_t c = std::max<int64_t>(n + n / 4, 1 << 16);
    hipStreamSynchronize(s->stream);
    hipFree(s->k0); hipFree(s->k1); hipFree(s->v0); hipFree(s->v1); hipFree(s->r0); hipFree(s->r1);
    hipFree(s->scratch);
    SCHECK(hipMalloc((void**)&s->k0, c * 8));
    SCHECK(hipMalloc((void**)&s->k1, c * 8));
    SCHECK(hipMalloc((void**)&s->v0, c * 4));
    SCHECK(hipMalloc((void**)&s->v1, c * 4));
    SCHECK(hipMalloc((void**)&s->r0, c * 4));
    SCHECK(hipMalloc((void**)&s->r1, c * 4));
    SCHECK(hipMalloc((void**)&s->scratch, radix_sort_scratch_bytes(c)));
    s->buf_cap = c;
    return GW_OK;
}

static int rehash_sess(SessionState* s, int64_t new_cap, std::string& err) {
    TableView nt;
    int rc = alloc_sess_table(s, nt, new_cap, s->tv.ring, err);
    if (rc) return rc;
    SCHECK(launch_status_set(s->d_st, 0, 0, 1, s->stream));  // zero sh[].ins (used slots)
    if (s->count_mode)
        hipLaunchKernelGGL(k_cnt_rehash, dim3(grid_of(s->tv.cap + 1)), dim3(256), 0, s->stream, s->tv, nt, s->d_st);
    else
        hipLaunchKernelGGL(k_sess_rehash, dim3(grid_of(s->tv.cap + 1)), dim3(256), 0, s->stream, s->tv, nt, s->d_st);
    SCHECK(hipGetLastError());
    SCHECK(hipStreamSynchronize(s->stream));
    hipFree(s->tv.base);
    s->tv = nt;
    s->stats.rehashes++;
    return session_refresh(s, err);
}

static int widen(SessionState* s, int newK, std::string& err) {
    TableView nt;
    int rc = alloc_sess_table(s, nt, s->tv.cap, newK, err);
    if (rc) return rc;
    hipLaunchKernelGGL(k_sess_rewiden, dim3(grid_of(s->tv.cap + 1)), dim3(256), 0, s->stream, s->tv, nt);
    SCHECK(hipGetLastError());
    SCHECK(hipStreamSynchronize(s->stream));
    hipFree(s->tv.base);
    s->tv = nt;
    return GW_OK;
}

static int ensure_rows(SessionState* s, int64_t need, std::string& err) {
    if (need <= s->o_cap) return GW_OK;
    const int64_t before = (int64_t)s->h_st->rows;
    const int64_t c = std::max<int64_t>(need + need / 4, 1 << 16);
    int64_t* nb[4];
    for (int q = 0; q < 4; ++q) SCHECK(hipMalloc((void**)&nb[q], c * 8));
    int64_t* old[4] = {s->o_key, s->o_start, s->o_end, s->o_res};
    for (int q = 0; q < 4; ++q) {
        if (old[q] && before) SCHECK(hipMemcpyAsync(nb[q], old[q], before * 8, hipMemcpyDeviceToDevice, s->stream));
    }
    SCHECK(hipStreamSynchronize(s->stream));
    for (int q = 0; q < 4; ++q) hipFree(old[q]);
    s->o_key = nb[0]; s->o_start = nb[1]; s->o_end = nb[2]; s->o_res = nb[3];
    s->o_cap = c;
    return GW_OK;
}

static int ensure_late(SessionState* s, int64_t need, std::string& err) {
    if (need <= s->lo_cap) return GW_OK;
    const int64_t used = (int64_t)s->h_st->n_late_out;  // exact: the session path is synchronous
    const int64_t c = std::max<int64_t>(need + need / 2, 1 << 16);
    for (int q = 0; q < 3; ++q) {
        int64_t* nb;
        SCHECK(hipMalloc((void**)&nb, c * 8));
        if (s->lo_buf[q] && used) SCHECK(hipMemcpyAsync(nb, s->lo_buf[q], used * 8, hipMemcpyDeviceToDevice, s->stream));
        SCHECK(hipStreamSynchronize(s->stream));
        hipFree(s->lo_buf[q]);
        s->lo_buf[q] = nb;
    }
    s->lo_cap = c;
    return GW_OK;
}

int session_pending_late(SessionState* s, int64_t* n, std::string& err) {
    int rc = session_refresh(s, err);
    if (rc) return rc;
    *n = (int64_t)s->h_st->n_late_out - s->lo_head;
    return GW_OK;
}

int session_drain_late(SessionState* s, int64_t* key, int64_t* ts, int64_t* val, int64_t cap, int64_t* n,
                       std::string& err) {
    int64_t pending;
    int rc = session_pending_late(s, &pending, err);
    if (rc) return rc;
    const int64_t c = std::min(cap, pending), o = s->lo_head;
    int64_t* dst[3] = {key, ts, val};
    for (int q = 0; q < 3 && c > 0; ++q)
        if (dst[q]) SCHECK(hipMemcpyAsync(dst[q], s->lo_buf[q] + o, c * 8, hipMemcpyDeviceToHost, s->stream));
    SCHECK(hipStreamSynchronize(s->stream));
    *n = c;
    s->lo_head += c;
    if (c == pending) {
        s->lo_head = 0;
        if ((rc = set_word(s, offsetof(DevStatus, n_late_out), 0, err))) return rc;
    }
    return c < pending ? GW_E_OUTPUT_FULL : GW_OK;
}

// Count windows: slot per record, stable grouping by slot, one in-order fold per key.
static int count_ingest(SessionState* s, int64_t n, const int64_t* key, const int64_t* val, std::string& err) {
    int rc;
    if ((rc = session_refresh(s, err))) return rc;
    if (n <= 0) return GW_OK;
    if ((int64_t)n > (int64_t)0xffffffffLL) { err = "batch too large"; return GW_E_INVALID; }
    if ((double)(s->h_st->used_slots + n) > 0.7 * (double)s->tv.cap) {
        int64_t want = s->tv.cap;
        while ((double)(s->h_st->used_slots + n) > 0.7 * (double)want) want *= 2;
        if ((rc = rehash_sess(s, want, err))) return rc;
    }
    if ((rc = ensure_bufs(s, n, err))) return rc;
    // every element fires at most one window
    if ((rc = ensure_rows(s, (int64_t)s->h_st->rows + n, err))) return rc;
    int slot_bits = 1;
    while (slot_bits < 63 && ((uint64_t)(s->tv.cap + 1) >> slot_bits)) ++slot_bits;
    auto ev = s->timing ? get_ev(s) : std::pair<hipEvent_t, hipEvent_t>{};
    if (s->timing) SCHECK(hipEventRecord(ev.first, s->stream));
    hipLaunchKernelGGL(k_cnt_slot, dim3(grid_of(n)), dim3(256), 0, s->stream, s->tv, key, n, s->k0, s->v0, s->d_st);
    SCHECK(hipGetLastError());
    int alt = 0;
    SCHECK(radix_sort_pairs(s->k0, s->v0, s->k1, s->v1, n, slot_bits, s->scratch, s->stream, &alt));
    const uint64_t* ks = alt ? s->k1 : s->k0;
    const uint32_t* perm = alt ? s->v1 : s->v0;
#define L(A)                                                                                             \
    hipLaunchKernelGGL(k_cnt_apply<A>, dim3(grid_of(n)), dim3(256), 0, s->stream, s->tv, s->cg, ks, perm, n, \
                       s->cfg.agg == GW_COUNT ? nullptr : val, s->o_key, s->o_start, s->o_end, s->o_res, s->d_st)
    GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
    SCHECK(hipGetLastError());
    if (s->timing) {
        SCHECK(hipEventRecord(ev.second, s->stream));
        s->ev_pending[0].push_back(ev);
    }
    if ((rc = session_refresh(s, err))) return rc;
    if (s->h_st->flags & GW_DF_TABLE_FULL) { err = "count-window state table overflow"; return GW_E_OOM; }
    return GW_OK;
}

int session_ingest(SessionState* s, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val, int64_t wm,
                   std::string& err) {
    if (s->count_mode) return count_ingest(s, n, key, val, err);
    int rc;
    if ((rc = session_refresh(s, err))) return rc;
    if (n <= 0) return GW_OK;
    if ((int64_t)n > (int64_t)0xffffffffLL) { err = "batch too large"; return GW_E_INVALID; }
    // keep the linear-probing load below 0.7 (worst case: every record a new key)
    if ((double)s->h_st->used_slots > 0.7 * (double)s->tv.cap ||
        (double)(s->h_st->used_slots + n) > 0.95 * (double)s->tv.cap) {
        int64_t want = s->tv.cap;
        while ((double)(s->h_st->used_slots + n) > 0.7 * (double)want) want *= 2;
        if ((rc = rehash_sess(s, want, err))) return rc;
    }
    if ((rc = ensure_bufs(s, n, err))) return rc;
    const long long init_mm[2] = {INT64_MAX, INT64_MIN};
    SCHECK(hipMemcpyAsync(s->d_mm, init_mm, 16, hipMemcpyHostToDevice, s->stream));
    hipLaunchKernelGGL(k_sess_minmax, dim3(grid_of(n)), dim3(256), 0, s->stream, ts, n, s->d_mm, s->d_st);
    long long mm[2];
    SCHECK(hipMemcpyAsync(mm, s->d_mm, 16, hipMemcpyDeviceToHost, s->stream));
    if ((rc = session_refresh(s, err))) return rc;
    const uint64_t span = (uint64_t)mm[1] - (uint64_t)mm[0];
    int ts_bits = 1;
    while (ts_bits < 64 && (span >> ts_bits)) ++ts_bits;
    int slot_bits = 1;
    while (slot_bits < 63 && ((uint64_t)(s->tv.cap) >> slot_bits)) ++slot_bits;
    if (ts_bits + slot_bits > 64) {
        err = "session batch spans too many milliseconds for the (slot, ts) sort key";
        return GW_E_UNSUPPORTED;
    }
    auto ev = s->timing ? get_ev(s) : std::pair<hipEvent_t, hipEvent_t>{};
    if (s->timing) SCHECK(hipEventRecord(ev.first, s->stream));
    for (int attempt = 0;; ++attempt) {
        hipLaunchKernelGGL(k_sess_prep, dim3(grid_of(n)), dim3(256), 0, s->stream, key, ts, n, (int64_t)mm[0], ts_bits,
                           s->tv, s->k0, s->v0, s->d_st);
        if ((rc = session_refresh(s, err))) return rc;
        if (!(s->h_st->flags & GW_DF_TABLE_FULL)) break;
        if (attempt > 4) { err = "session state table full"; return GW_E_OOM; }
        SCHECK(launch_status_set(s->d_st, 0, 0, 2, s->stream));  // zero sh[].flags
        if ((rc = rehash_sess(s, s->tv.cap * 2, err))) return rc;
        slot_bits++;
        if (ts_bits + slot_bits > 64) { err = "session sort key overflow"; return GW_E_UNSUPPORTED; }
    }
    int alt = 0;
    SCHECK(radix_sort_pairs(s->k0, s->v0, s->k1, s->v1, n, ts_bits + slot_bits, s->scratch, s->stream, &alt));
    SegArgs a{};
    a.skey = alt ? s->k1 : s->k0;
    a.perm = alt ? s->v1 : s->v0;
    a.n = n;
    a.ts_bits = ts_bits;
    a.ts_min = mm[0];
    a.val = val;
    a.gap = s->cfg.gap;
    a.wm = wm;
    a.lateness = s->cfg.allowed_lateness;
    a.purge = a.lateness > 0 && s->cfg.trigger == GW_PURGING_EVENT_TIME_TRIGGER;
    a.st = s->d_st;
    if (a.lateness > 0) {  // an element fires at most one window at once
        if ((rc = ensure_rows(s, (int64_t)s->h_st->rows + n, err))) return rc;
        a.o_key = s->o_key; a.o_start = s->o_start; a.o_end = s->o_end; a.o_res = s->o_res;
    }
    a.ts = ts;
    a.key = key;
    if (s->cfg.flags & GW_FLAG_LATE_SIDE_OUTPUT) {
        if ((rc = ensure_late(s, (int64_t)s->h_st->n_late_out + n, err))) return rc;
        a.lo_key = s->lo_buf[0]; a.lo_ts = s->lo_buf[1]; a.lo_val = s->lo_buf[2];
    }
    uint32_t* rin = s->r0;
    uint32_t* rout = s->r1;
    int64_t n_retry = 0;
    for (int pass = 0;; ++pass) {
        if ((rc = set_word(s, offsetof(DevStatus, overflow), 0, err))) return rc;
        if ((rc = set_word(s, offsetof(DevStatus, pad[1]), 0, err))) return rc;
        a.t = s->tv;
        a.retry_in = pass ? rin : nullptr;
        a.n_retry_in = n_retry;
        a.retry_out = rout;
        const unsigned g = pass ? grid_of(n_retry) : grid_of(n);
#define L(A) hipLaunchKernelGGL(k_sess_segment<A>, dim3(g), dim3(256), 0, s->stream, a)
        GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
        SCHECK(hipGetLastError());
        if ((rc = session_refresh(s, err))) return rc;
        if (!s->h_st->overflow) break;
        const unsigned long long need = s->h_st->pad[1];
        if (need > (unsigned long long)kMaxLocalSess || pass > 8) {
            err = "more than 32 in-flight sessions for one key in one batch is not supported on the GPU path";
            return GW_E_UNSUPPORTED;
        }
        int newK = s->tv.ring;
        while ((unsigned long long)newK < need) newK *= 2;
        if (newK > kMaxLocalSess) newK = kMaxLocalSess;
        if ((rc = widen(s, newK, err))) return rc;
        n_retry = (int64_t)s->h_st->overflow;
        std::swap(rin, rout);
    }
    if (s->timing) {
        SCHECK(hipEventRecord(ev.second, s->stream));
        s->ev_pending[0].push_back(ev);
    }
    return GW_OK;
}

int session_fire(SessionState* s, int64_t wm, int64_t* fired, std::string& err) {
    if (s->count_mode) {  // GlobalWindows: event time fires nothing (CountTrigger.onEventTime: CONTINUE)
        s->wm = wm;
        *fired = 0;
        return GW_OK;
    }
    int rc;
    if ((rc = session_refresh(s, err))) return rc;
    const int64_t before = (int64_t)s->h_st->rows;
    const int64_t need = before + (int64_t)(s->h_st->used_slots + 1) * s->tv.ring;
    if (need > s->o_cap) {
        const int64_t c = std::max<int64_t>(need + need / 4, 1 << 16);
        int64_t* nb[4];
        for (int q = 0; q < 4; ++q) SCHECK(hipMalloc((void**)&nb[q], c * 8));
        int64_t* old[4] = {s->o_key, s->o_start, s->o_end, s->o_res};
        for (int q = 0; q < 4; ++q) {
            if (old[q] && before) SCHECK(hipMemcpyAsync(nb[q], old[q], before * 8, hipMemcpyDeviceToDevice, s->stream));
        }
        SCHECK(hipStreamSynchronize(s->stream));
        for (int q = 0; q < 4; ++q) hipFree(old[q]);
        s->o_key = nb[0]; s->o_start = nb[1]; s->o_end = nb[2]; s->o_res = nb[3];
        s->o_cap = c;
    }
    auto ev = s->timing ? get_ev(s) : std::pair<hipEvent_t, hipEvent_t>{};
    if (s->timing) SCHECK(hipEventRecord(ev.first, s->stream));
    const unsigned fg = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(1, (s->tv.cap + 1 + 255) / 256));
#define L(A)                                                                                               \
    hipLaunchKernelGGL(k_sess_fire<A>, dim3(fg), dim3(256), 0, s->stream, s->tv, wm, s->cfg.allowed_lateness, \
                       (int)(s->cfg.allowed_lateness > 0 && s->cfg.trigger == GW_PURGING_EVENT_TIME_TRIGGER), \
                       s->o_key, s->o_start, s->o_end, s->o_res, s->d_st)
    GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
    SCHECK(hipGetLastError());
    if (s->timing) {
        SCHECK(hipEventRecord(ev.second, s->stream));
        s->ev_pending[1].push_back(ev);
    }
    s->stats.fires++;
    if ((rc = session_refresh(s, err))) return rc;
    *fired = (int64_t)s->h_st->rows - before;
    s->wm = wm;
    return GW_OK;
}

void session_rows(SessionState* s, int64_t** k, int64_t** st, int64_t** en, int64_t** r, int64_t* total) {
    *k = s->o_key; *st = s->o_start; *en = s->o_end; *r = s->o_res;
    *total = (int64_t)s->h_st->rows;
}

int session_clear_rows(SessionState* s, std::string& err) { return set_word(s, offsetof(DevStatus, rows), 0, err); }

// ---- snapshot / restore of in-flight sessions (gw_snapshot / gw_restore) -------------
// The heap backend snapshots, per key group, every (key, window) state entry plus the
// MergingWindowSet mapping (HeapSnapshotStrategy.java:97-154, MergingWindowSet.java:
// 95-104 persistState); in-flight sessions are exactly that state here, one
// (key, start, end, a0, a1) entry per session.
int session_collect(SessionState* s, int32_t kg_lo, int32_t kg_hi, std::vector<int64_t>& ent,
                    std::vector<int32_t>& kgs, std::string& err) {
    SCHECK(hipStreamSynchronize(s->stream));
    const TableView& t = s->tv;
    const size_t words = (size_t)(t.cap + 1) * t.stride_w;
    std::vector<int64_t> h(words);
    SCHECK(hipMemcpy(h.data(), t.base, words * 8, hipMemcpyDeviceToHost));
    const int SW = t.words;
    for (int64_t i = 0; i <= t.cap; ++i) {
        const int64_t* sp = h.data() + (size_t)i * t.stride_w;
        if (sp[1] == 0) continue;
        const int64_t key = i == t.cap ? kEmptyKey : sp[0];
        const int32_t kg = key_group_for_hash(java_long_hash(key), s->cfg.max_parallelism);
        if (kg < kg_lo || kg > kg_hi) continue;
        if (s->count_mode) {  // (key, element count, ring of pane accumulators)
            ent.push_back(key);
            ent.insert(ent.end(), sp + 1, sp + 2 + t.ring * SW);
            kgs.push_back(kg);
            continue;
        }
        const int cnt = (int)(uint32_t)(uint64_t)sp[1];
        for (int q = 0; q < cnt; ++q) {
            const int64_t* x = sp + 2 + q * SW;
            const int64_t fired = (int64_t)(((uint64_t)sp[1] >> (32 + q)) & 1ull);  // kept under allowed lateness
            const int64_t e[6] = {key, x[0], x[1], x[2], SW == 4 ? x[3] : 0, fired};
            ent.insert(ent.end(), e, e + 6);
            kgs.push_back(kg);
        }
    }
    return GW_OK;
}

int session_entry_words(SessionState* s) { return s->count_mode ? 2 + s->tv.ring * s->tv.words : 6; }

static int count_restore(SessionState* s, const int64_t* ent, int64_t n, std::string& err) {
    int rc;
    if ((double)(s->h_st->used_slots + n) > 0.7 * (double)s->tv.cap) {
        int64_t want = s->tv.cap;
        while ((double)(s->h_st->used_slots + n) > 0.7 * (double)want) want *= 2;
        if ((rc = rehash_sess(s, want, err))) return rc;
    }
    const int64_t bytes = n * session_entry_words(s) * 8;
    int64_t* d = nullptr;
    SCHECK(hipMalloc((void**)&d, bytes));
    SCHECK(hipMemcpy(d, ent, bytes, hipMemcpyHostToDevice));
    if ((rc = set_word(s, offsetof(DevStatus, overflow), 0, err))) return rc;
    hipLaunchKernelGGL(k_cnt_restore, dim3(grid_of(n)), dim3(256), 0, s->stream, s->tv, d, n, s->d_st);
    SCHECK(hipGetLastError());
    rc = session_refresh(s, err);
    hipFree(d);
    if (rc) return rc;
    if (s->h_st->flags & GW_DF_TABLE_FULL) { err = "count-window state table overflow"; return GW_E_OOM; }
    if (s->h_st->overflow) {
        err = "a restored key already holds count-window state in this operator";
        return GW_E_UNSUPPORTED;
    }
    return GW_OK;
}

int session_restore(SessionState* s, const int64_t* ent, int64_t n, std::string& err) {
    int rc;
    if ((rc = session_refresh(s, err))) return rc;
    if (n <= 0) return GW_OK;
    if (s->count_mode) return count_restore(s, ent, n, err);
    std::vector<int64_t> ord(n);
    for (int64_t i = 0; i < n; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
        const int64_t* x = ent + a * 6;
        const int64_t* y = ent + b * 6;
        return x[0] != y[0] ? x[0] < y[0] : x[1] < y[1];
    });
    std::vector<int64_t> rk, roff, rs;
    rs.reserve((size_t)n * 5);
    int maxk = 0, run = 0;
    for (int64_t j = 0; j < n; ++j) {
        const int64_t* x = ent + ord[j] * 6;
        if (j == 0 || x[0] != rk.back()) {
            rk.push_back(x[0]);
            roff.push_back(j);
            run = 0;
        }
        maxk = std::max(maxk, ++run);
        rs.insert(rs.end(), x + 1, x + 6);
    }
    roff.push_back(n);
    const int64_t nk = (int64_t)rk.size();
    if (maxk > kMaxLocalSess) {
        err = "more than 32 in-flight sessions for one key is not supported on the GPU path";
        return GW_E_UNSUPPORTED;
    }
    if (maxk > s->tv.ring) {
        int newK = s->tv.ring;
        while (newK < maxk) newK *= 2;
        if ((rc = widen(s, std::min(newK, kMaxLocalSess), err))) return rc;
    }
    if ((double)(s->h_st->used_slots + nk) > 0.7 * (double)s->tv.cap) {
        int64_t want = s->tv.cap;
        while ((double)(s->h_st->used_slots + nk) > 0.7 * (double)want) want *= 2;
        if ((rc = rehash_sess(s, want, err))) return rc;
    }
    int64_t *d_k = nullptr, *d_o = nullptr, *d_s = nullptr;
    SCHECK(hipMalloc((void**)&d_k, nk * 8));
    SCHECK(hipMalloc((void**)&d_o, (nk + 1) * 8));
    SCHECK(hipMalloc((void**)&d_s, n * 40));
    SCHECK(hipMemcpy(d_k, rk.data(), nk * 8, hipMemcpyHostToDevice));
    SCHECK(hipMemcpy(d_o, roff.data(), (nk + 1) * 8, hipMemcpyHostToDevice));
    SCHECK(hipMemcpy(d_s, rs.data(), n * 40, hipMemcpyHostToDevice));
    if ((rc = set_word(s, offsetof(DevStatus, overflow), 0, err))) return rc;
#define L(A) \
    hipLaunchKernelGGL(k_sess_restore<A>, dim3(grid_of(nk)), dim3(256), 0, s->stream, s->tv, d_k, d_o, d_s, nk, s->d_st)
    GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
    SCHECK(hipGetLastError());
    rc = session_refresh(s, err);
    hipFree(d_k);
    hipFree(d_o);
    hipFree(d_s);
    if (rc) return rc;
    if (s->h_st->flags & GW_DF_TABLE_FULL) { err = "session state table full"; return GW_E_OOM; }
    if (s->h_st->overflow) {
        err = "restored sessions and in-flight sessions of one key exceed the slot's session list";
        return GW_E_UNSUPPORTED;
    }
    return GW_OK;
}

int64_t session_late(SessionState* s) { return (int64_t)s->h_st->late; }

void session_stats(SessionState* s, gw_stats* out) {
    out->late_dropped = (int64_t)s->h_st->late;
    out->live_keys = (int64_t)s->h_st->used_slots;
    out->table_capacity = s->tv.cap;
    out->table_bytes = (int64_t)(s->tv.cap + 1) * s->tv.stride_w * 8;
    out->session_merges = (int64_t)s->h_st->merges;
    out->fires = s->stats.fires;
    out->rehashes = s->stats.rehashes;
}

void session_enable_timing(SessionState* s, bool on) { s->timing = on; }

int session_kernel_time(SessionState* s, int which, double* ms, int64_t* launches) {
    hipStreamSynchronize(s->stream);
    resolve_timers(s);
    const int w = which ? 1 : 0;
    if (ms) *ms = s->t_count[w] ? s->t_total[w] / (double)s->t_count[w] : 0.0;
    if (launches) *launches = s->t_count[w];
    s->t_total[w] = 0;
    s->t_count[w] = 0;
    return GW_OK;
}

}  // namespace gw
