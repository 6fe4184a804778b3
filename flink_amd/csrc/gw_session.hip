// gw_session.hip — event-time session windows (gap merge) and count windows on gfx950.
//
// Reference semantics (paths relative to the Flink tree):
//   EventTimeSessionWindows.assignWindows -> [ts, ts + gap)
//     (flink-streaming-java/.../api/windowing/assigners/EventTimeSessionWindows.java:61-64)
//   TimeWindow.intersects (inclusive: touching windows merge) / cover / mergeWindows
//     (RS/api/windowing/windows/TimeWindow.java:116-123,208-254)
//   MergingWindowSet.addWindow (RS/runtime/operators/windowing/MergingWindowSet.java:153-224)
//   WindowOperator.processElement merging branch incl. "drop if the window is already
//     late" (RS/runtime/operators/windowing/WindowOperator.java:303-403, 440-446)
//   AbstractHeapMergingState.mergeNamespaces (RR/state/heap/AbstractHeapMergingState.java:65-91)
//   EventTimeTrigger + onEventTime: a session fires once when end-1 <= watermark.
//
// MI355X design: per watermark batch every record finds its key's slot,
// a stable radix sort by slot (rocPRIM) groups each key's records in ARRIVAL order, and one
// thread per key replays them through MergingWindowSet.addWindow semantics -- the
// reference's own record-at-a-time order, so late records, immediate firings and merges
// behave exactly as in the reference, with no separate replay path.  The thread keeps the
// key's in-flight sessions in its LDS lane (kLaneSess sessions); a key's sessions live
// inline in its slot of the main table (K1 = 2 / 3 per slot).  A key with more in-flight
// sessions moves to the wide table (one slot per such key, K2 sessions each, K2 doubled as
// needed): its runs are replayed there in global memory.  No per-key session limit.
#include "gw_kernels.h"
#include "gw_session.h"
#include "gw_sort.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

// The slot sort's rocPRIM configuration: 9 bits per onesweep pass, so 12.5M keys' 26 slot
// bits take 3 passes instead of the library default's 4 at 8 bits (sessions config 7.4 ->
// 8.5 G events/s; 10 and 11 bits measured slower, profiles/r3/experiments.txt).
// GW_SESS_RADIX_BITS=0 builds the library default.
#ifndef GW_SESS_RADIX_BITS
#define GW_SESS_RADIX_BITS 9
#endif
#ifndef GW_SESS_SORT_ITEMS
#define GW_SESS_SORT_ITEMS 8
#endif
#if GW_SESS_RADIX_BITS
using SlotSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, GW_SESS_SORT_ITEMS>,
                                        GW_SESS_RADIX_BITS, rocprim::block_radix_rank_algorithm::match>>;
#else
using SlotSortConfig = rocprim::default_config;
#endif


namespace gw {

constexpr int kLaneSess = 3;        // sessions a thread replays in LDS
constexpr int kSegThreads = 128;
constexpr int kWideWords = 5;       // wide-table session: start, end, a0, a1, fired
constexpr uint64_t kBigMeta = 1ull << 31;  // main-table slot word 1: the key lives in the wide table
constexpr uint64_t kPuntMeta = 1ull << 30; // ... the key's later records of this batch go to the punt list

struct SegArgs {
    const uint32_t* slot;   // sorted main-table slot of each record
    const uint32_t* perm;   // its arrival index (stable sort: arrival order within a slot)
    int64_t n;
    const int64_t* key;
    const int64_t* ts;
    const int64_t* val;
    const int64_t* rec;     // (ts, value) per record in arrival order, 16-B aligned: one gather per record
    int64_t gap;
    int64_t wm;             // current watermark (all records of the batch see it)
    int64_t lateness;       // allowed lateness (WindowOperator.allowedLateness)
    int purge;              // PurgingTrigger: a fired session keeps an empty state until cleanup
    int64_t* o_key;         // rows of windows an element fires at once (EventTimeTrigger.onElement
    int64_t* o_start;       //   FIRE: window max timestamp <= watermark; lateness > 0 only)
    int64_t* o_end;
    int64_t* o_res;
    int64_t* lo_key;        // late side output (GW_FLAG_LATE_SIDE_OUTPUT), append at st->n_late_out
    int64_t* lo_ts;
    int64_t* lo_val;
    TableView t;            // main table: ring = K1 sessions per slot, words = words per session
    TableView w;            // wide table: ring = K2, words = kWideWords
    uint32_t* punt;         // main pass: runs for the wide table (append at st->overflow)
    int64_t* mig;           // main pass: finished lists of more than K1 sessions (append at st->pad[0])
    const uint32_t* runs;   // wide pass: run heads to replay
    int64_t n_runs;
    uint32_t* retry;        // wide pass: runs that did not fit K2 (append at st->overflow)
    DevStatus* st;
    int gshift;             // records are grouped by slot >> gshift (the sort skips the low bits)
    // region-partitioned ingest (k_sp_part / k_sp_group / k_sp_keys)
    const int64_t* p_key;   // pass-1 output, tile-major, bucket runs inside each tile: keys
    const longlong2* p_tv;  //   and (timestamp, value) pairs
    const uint32_t* col;    // [bucket][tile] run descriptors (start << 16 | count)
    int64_t ntiles;
    int lcap, bb;           // log2(table capacity), bucket bits (bucket = home >> (lcap - bb))
    int exp;                // GW_SP_EXP: measurement variants of k_sp_keys (0: none)
    uint32_t* slow;         // home slots for k_sp_slow (bucket << 14 | head), append at st->spills
    int64_t* pu_key;        // punted records (arrival order per key), append at st->overflow
    int64_t* pu_ts;
    int64_t* pu_val;
};

struct Sess {
    int64_t s, e, a0, a1;
    int64_t f;  // its event-time timer has fired (kept for allowed lateness until cleanup)
};

// Main-table slot word 1: in-flight session count (low 31 bits), kBigMeta, fired bit per
// session (high 32 bits).
__device__ __forceinline__ int slot_cnt(int64_t w) { return (int)((uint64_t)w & 0x3fffffffull); }
__device__ __forceinline__ bool slot_big(int64_t w) { return ((uint64_t)w & kBigMeta) != 0; }
__device__ __forceinline__ bool slot_fired(int64_t w, int q) { return ((uint64_t)w >> (32 + q)) & 1ull; }

// WindowOperator.cleanupTime (:670-677, overflow -> Long.MAX_VALUE, never cleaned) <= wm
__device__ __forceinline__ bool cleaned_at(int64_t end, int64_t lateness, int64_t wm) {
    const int64_t mx = end - 1;
    int64_t ct;
    if (__builtin_add_overflow(mx, lateness, &ct)) ct = INT64_MAX;
    return ct <= wm;
}

// The watermark at which a session needs the fire sweep: its timer (max timestamp) while it
// has not fired, its cleanup time once it has (kept for allowed lateness).
__device__ __forceinline__ int64_t due_time(int64_t end, bool fired, int64_t lateness) {
    const int64_t mx = end - 1;
    if (!fired) return mx;
    int64_t ct;
    if (__builtin_add_overflow(mx, lateness, &ct)) ct = INT64_MAX;
    return ct;
}

// Per slot, the earliest due time of its sessions (INT64_MAX: none, or the key lives in the
// wide table), in a dense array after the slots: the fire sweep reads 8 bytes per slot and
// touches only the slots with something due.
__device__ __forceinline__ int64_t* due_of(const TableView& t) { return t.base + (t.cap + 1) * (int64_t)t.stride_w; }

__device__ __forceinline__ int64_t inline_due(const int64_t* sp, int SW, int64_t lateness) {
    const int64_t w1 = sp[1];
    if (slot_big(w1)) return INT64_MAX;
    int64_t m = INT64_MAX;
    for (int q = 0, c = slot_cnt(w1); q < c; ++q) m = min(m, due_time(sp[2 + q * SW + 1], slot_fired(w1, q), lateness));
    return m;
}
__device__ __forceinline__ int64_t wide_due(const int64_t* sp, int64_t lateness) {
    int64_t m = INT64_MAX;
    for (int q = 0, c = (int)sp[1]; q < c; ++q) {
        const int64_t* x = sp + 2 + q * kWideWords;
        m = min(m, due_time(x[1], x[4] != 0, lateness));
    }
    return m;
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

// A session list (sorted by start, disjoint) in LDS or in a wide-table slot: SoA with a
// stride between fields, so both live in the same code.
struct SessList {
    int64_t* p;     // field f of session q at p[f * fs + q * qs]
    int fs, qs;
};
__device__ __forceinline__ Sess sl_get(const SessList& l, int q) {
    const int64_t* x = l.p + q * l.qs;
    return Sess{x[0], x[l.fs], x[2 * l.fs], x[3 * l.fs], x[4 * l.fs]};
}
__device__ __forceinline__ void sl_put(const SessList& l, int q, const Sess& v) {
    int64_t* x = l.p + q * l.qs;
    x[0] = v.s; x[l.fs] = v.e; x[2 * l.fs] = v.a0; x[3 * l.fs] = v.a1; x[4 * l.fs] = v.f;
}

// MergingWindowSet.addWindow + WindowOperator.processElement (merging branch) for one
// element: the window [ts, ts + gap) merges with every session it intersects (inclusive);
// a window that merges with nothing and is already late is skipped (late: counted or sent
// to the side output); a merged or new window whose max timestamp <= watermark fires at
// once (EventTimeTrigger.onElement FIRE; PurgingTrigger purges), otherwise its timer is
// (re-)armed.  Returns false if a new session does not fit `cap`.  `dry`: no rows and no
// side output are written (a trial replay that may be abandoned).
template <int AGG>
__device__ __forceinline__ bool add_element_tv(const SegArgs& a, const SessList& l, int& cnt, int cap, int64_t key,
                                               int64_t ts, int64_t value, unsigned long long& late,
                                               unsigned long long& merges, unsigned long long& flags, bool dry) {
    struct { int64_t ts, v; } tv{ts, value};
    int64_t we;
    if (__builtin_add_overflow(ts, a.gap, &we)) { flags |= GW_DF_RANGE; return true; }
    const int64_t ws = ts;
    int lo = -1, hi = -1;
    for (int q = 0; q < cnt; ++q) {
        const int64_t s = l.p[q * l.qs], e = l.p[l.fs + q * l.qs];
        if (s <= we && e >= ws) {
            if (lo < 0) lo = q;
            hi = q;
        }
    }
    int64_t c0, c1;
    record_cell(AGG, tv.v, c0, c1);
    if (lo < 0) {
        if (cleaned_at(we, a.lateness, a.wm)) {  // isWindowLate: skipped; the element is late
            if (!a.lo_key) {
                late++;
            } else if (!dry) {  // sideOutput(element) (WindowOperator.java:440-446, 587-588)
                const unsigned long long o = atomicAdd(&a.st->n_late_out, 1ull);
                a.lo_key[o] = key;
                a.lo_ts[o] = ts;
                a.lo_val[o] = tv.v;
            }
            return true;
        }
        if (cnt == cap) return false;
        int q = cnt;
        while (q > 0 && l.p[(q - 1) * l.qs] > ws) {
            sl_put(l, q, sl_get(l, q - 1));
            --q;
        }
        Sess x{ws, we, c0, c1, (int64_t)(we - 1 <= a.wm)};
        if (x.f) {  // onElement: FIRE (PurgingTrigger: FIRE_AND_PURGE)
            if (!dry) emit_now<AGG>(a, key, x);
            if (a.purge) purge_acc<AGG>(x.a0, x.a1);
        }
        sl_put(l, q, x);
        cnt++;
        return true;
    }
    Sess m = sl_get(l, lo);
    if (ws < m.s) m.s = ws;
    for (int q = lo + 1; q <= hi; ++q) {
        const Sess y = sl_get(l, q);
        if (y.e > m.e) m.e = y.e;
        fold_cell(AGG, m.a0, m.a1, y.a0, y.a1);
        merges++;
    }
    if (we > m.e) m.e = we;
    fold_cell(AGG, m.a0, m.a1, c0, c1);
    m.f = m.e - 1 <= a.wm;  // onElement FIRE, or onMerge registers the merged window's timer
    if (m.f) {
        if (!dry) emit_now<AGG>(a, key, m);
        if (a.purge) purge_acc<AGG>(m.a0, m.a1);
    }
    sl_put(l, lo, m);
    const int removed = hi - lo;
    for (int q = hi + 1; q < cnt; ++q) sl_put(l, q - removed, sl_get(l, q));
    cnt -= removed;
    return true;
}

// The same for element `idx` of the batch, read from the (ts, value) pairs of k_sess_prep.
template <int AGG>
__device__ __forceinline__ bool add_element(const SegArgs& a, const SessList& l, int& cnt, int cap, int64_t key,
                                            int64_t idx, unsigned long long& late, unsigned long long& merges,
                                            unsigned long long& flags, bool dry = false) {
    struct alignas(16) TsVal { int64_t ts, v; };
    const TsVal tv = reinterpret_cast<const TsVal*>(a.rec)[idx];
    return add_element_tv<AGG>(a, l, cnt, cap, key, tv.ts, tv.v, late, merges, flags, dry);
}

// Main pass: one thread per key's run.  The run's elements replay against the key's
// inline sessions in the thread's LDS lane.  A run that could need more than kLaneSess
// sessions is first replayed dry (no rows, no side output); only if the list really
// outgrows the lane, or the key is already in the wide table, does it go to the wide pass.
// Without allowed lateness and side output a replay has no effects beyond the slot, so
// the dry replay is the real one.
// One key's records among the group [i, j) (those whose slot is `slot`, L of them, the first
// at i), in arrival order.
template <int AGG>
__device__ __forceinline__ void seg_slot(const SegArgs& a, const SessList& l, int64_t i, int64_t j, uint32_t slot,
                                         int64_t L, unsigned long long& late, unsigned long long& merges,
                                         unsigned long long& flags) {
    int64_t* sp = slot_ptr(a.t, (int64_t)slot);
    const int64_t w1 = sp[1];
    const int SW = a.t.words;
    const int64_t key = sp[0];  // the sentinel slot's key word is Long.MIN_VALUE, its key
    bool ok = !slot_big(w1);
    bool dry = ok && slot_cnt(w1) + L > kLaneSess;  // could outgrow the lane
    const bool effects = a.lateness > 0 || a.lo_key;
    const unsigned long long l0 = late, m0 = merges;
    int cnt = 0;
    while (ok) {  // at most two replays: dry, then (with effects) the real one
        cnt = slot_cnt(w1);
        for (int q = 0; q < cnt; ++q) {
            const int64_t* x = sp + 2 + q * SW;
            sl_put(l, q, Sess{x[0], x[1], x[2], SW == 4 ? x[3] : 0, (int64_t)slot_fired(w1, q)});
        }
        // whole-slot groups (gshift 0): every record of [i, j) is the slot's, no slot re-read
        for (int64_t r = i; r < j && ok; ++r)
            if (a.gshift == 0 || a.slot[r] == slot)
                ok = add_element<AGG>(a, l, cnt, kLaneSess, key, a.perm[r], late, merges, flags, dry);
        if (!ok || !dry || !effects) break;
        dry = false;
        late = l0;
        merges = m0;
    }
    if (!ok) {
        late = l0;
        merges = m0;
        const unsigned long long at = atomicAdd(&a.st->overflow, 1ull);
        a.punt[at] = (uint32_t)i;  // the wide pass replays this slot's records from i to the group's end
        return;
    }
    if (cnt <= a.t.ring) {
        uint64_t fired = 0;
        int64_t due = INT64_MAX;
        for (int q = 0; q < cnt; ++q) {
            const Sess v = sl_get(l, q);
            int64_t* x = sp + 2 + q * SW;
            x[0] = v.s; x[1] = v.e; x[2] = v.a0;
            if (SW == 4) x[3] = v.a1;
            fired |= (uint64_t)(v.f != 0) << q;
            due = min(due, due_time(v.e, v.f != 0, a.lateness));
        }
        sp[1] = (int64_t)((fired << 32) | (uint64_t)(uint32_t)cnt);
        due_of(a.t)[slot] = due;
    } else {  // more sessions than the slot holds: the finished list moves to the wide table
        const unsigned long long at = atomicAdd(&a.st->pad[0], 1ull);
        int64_t* m = a.mig + at * (2 + kWideWords * kLaneSess);
        m[0] = (int64_t)slot;
        m[1] = cnt;
        for (int q = 0; q < cnt; ++q) {
            const Sess v = sl_get(l, q);
            int64_t* x = m + 2 + q * kWideWords;
            x[0] = v.s; x[1] = v.e; x[2] = v.a0; x[3] = v.a1; x[4] = v.f;
        }
        atomicMax(&a.st->pad[1], (unsigned long long)cnt);
    }
}

// Main pass: one thread per key's run.  The radix sort groups records by slot >> gshift
// (it skips the low bits: one pass fewer on large tables), so a group interleaves the runs
// of at most 2^gshift slots, each in arrival order.  A work item is the first record of a
// slot in its group; its thread replays that slot's records of the group against the
// key's inline sessions in its LDS lane.  A run that could need more than kLaneSess
// sessions is first replayed dry (no rows, no side output); only if the list really
// outgrows the lane, or the key is already in the wide table, does it go to the wide
// pass.  Without allowed lateness and side output a replay has no effects beyond the
// slot, so the dry replay is the real one.
__device__ __forceinline__ bool seg_is_item(const SegArgs& a, int64_t i) {
    if (i >= a.n) return false;
    if (i == 0) return true;
    const uint32_t slot = a.slot[i], grp = slot >> a.gshift;
    if ((a.slot[i - 1] >> a.gshift) != grp) return true;  // a group head
    for (int64_t q = i - 1; q >= 0; --q) {  // an earlier record of the slot in the group?
        const uint32_t x = a.slot[q];
        if (x == slot) return false;
        if ((x >> a.gshift) != grp) break;
    }
    return true;
}

template <int AGG>
__device__ __forceinline__ void seg_run(const SegArgs& a, const SessList& l, int64_t i, unsigned long long& late,
                                        unsigned long long& merges, unsigned long long& flags) {
    const uint32_t slot = a.slot[i], grp = slot >> a.gshift;
    int64_t j = i + 1, L = 1;
    for (; j < a.n; ++j) {
        const uint32_t x = a.slot[j];
        if ((x >> a.gshift) != grp) break;
        L += x == slot;
    }
    seg_slot<AGG>(a, l, i, j, slot, L, late, merges, flags);
}

// Each wave takes kSegChunk consecutive records, compacts their work items into LDS with
// ballots, and replays them 64 at a time: every lane owns a run (about one record in
// three starts one), not one lane per record.
constexpr int kSegChunk = 512;
template <int AGG>
__global__ void __launch_bounds__(kSegThreads) k_sess_segment(SegArgs a) {
    __shared__ int64_t lane[5 * kLaneSess * kSegThreads];
    __shared__ uint32_t heads[kSegThreads / 64][kSegChunk];
    const SessList l{lane + threadIdx.x, kLaneSess * kSegThreads, kSegThreads};
    unsigned long long late = 0, merges = 0, flags = 0;
    const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int64_t base = (blockIdx.x * (int64_t)(kSegThreads / 64) + w) * kSegChunk;
    int nh = 0;
    for (int c = 0; c < kSegChunk; c += 64) {
        const int64_t i = base + c + ln;
        const bool h = seg_is_item(a, i);
        const uint64_t b = __ballot(h);
        if (h) heads[w][nh + __popcll(b & ((1ull << ln) - 1ull))] = (uint32_t)(i - base);
        nh += __popcll(b);
    }
    __syncthreads();
    for (int q = ln; q < nh; q += 64) seg_run<AGG>(a, l, base + heads[w][q], late, merges, flags);
    late = wave_sum(late);
    merges = wave_sum(merges);
    flags = wave_ior(flags);
    if (ln == 0) {
        ShardCtr& sc = a.st->sh[blockIdx.x % kShards];
        if (late) atomicAdd(&sc.late, late);
        if (merges) atomicAdd(&sc.merges, merges);
        if (flags) atomicOr(&sc.flags, flags);
    }
}

// The key of main-table slot g moves to the wide table: a wide slot with its sessions.
__device__ __forceinline__ int64_t wide_slot_of(const TableView& w, int64_t key, unsigned long long& flags) {
    bool inserted;
    const int64_t g2 = find_or_insert(w, key, inserted);
    if (g2 < 0) flags |= GW_DF_TABLE_FULL;
    return g2;
}

// Finished lists of the main pass -> the wide table.
__global__ void __launch_bounds__(256) k_sess_migrate(TableView t, TableView w, const int64_t* mig, int64_t n,
                                                      int64_t lateness, DevStatus* st) {
    unsigned long long flags = 0, ins = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t* m = mig + i * (2 + kWideWords * kLaneSess);
        int64_t* sp = slot_ptr(t, m[0]);
        const int64_t key = m[0] == t.cap ? kEmptyKey : sp[0];
        bool inserted;
        const int64_t g2 = find_or_insert(w, key, inserted);
        if (g2 < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        ins += inserted;
        int64_t* d = slot_ptr(w, g2);
        const int cnt = (int)m[1];
        for (int x = 0; x < cnt * kWideWords; ++x) d[2 + x] = m[2 + x];
        d[1] = cnt;
        due_of(w)[g2] = wide_due(d, lateness);
        sp[1] = (int64_t)kBigMeta;
        due_of(t)[m[0]] = INT64_MAX;
    }
    flags = wave_ior(flags);
    ins = wave_sum(ins);
    if (__lane_id() == 0) {
        if (flags) atomicOr(&st->sh[blockIdx.x % kShards].flags, flags);
        if (ins) atomicAdd(&st->pad[2], ins);  // wide-table slots in use
    }
}

// Wide pass: one thread per punted run, against the key's wide slot in global memory.  A
// key not yet wide moves there first.  A run that could exceed K2 sessions is left for a
// retry after the host widens the table (nothing is written or emitted for it).
template <int AGG>
__global__ void __launch_bounds__(256) k_sess_wide(SegArgs a) {
    unsigned long long late = 0, merges = 0, flags = 0, ins = 0;
    for (int64_t r0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r0 < a.n_runs;
         r0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = a.runs[r0];  // the slot's first record in its group
        const uint32_t slot = a.slot[i];
        const uint32_t grp = slot >> a.gshift;
        int64_t j = i + 1, hi = a.n;  // sorted by group: the group ends at the first other group
        while (j < hi) {
            const int64_t mid = (j + hi) >> 1;
            if ((a.slot[mid] >> a.gshift) == grp) j = mid + 1; else hi = mid;
        }
        int64_t L = 0;
        for (int64_t q = i; q < j; ++q) L += a.slot[q] == slot;
        int64_t* sp = slot_ptr(a.t, (int64_t)slot);
        const int64_t key = (int64_t)slot == a.t.cap ? kEmptyKey : sp[0];
        bool inserted;
        const int64_t g2 = find_or_insert(a.w, key, inserted);
        if (g2 < 0) {
            flags |= GW_DF_TABLE_FULL;
            const unsigned long long at = atomicAdd(&a.st->overflow, 1ull);
            a.retry[at] = (uint32_t)i;
            continue;
        }
        ins += inserted;
        int64_t* d = slot_ptr(a.w, g2);
        const int64_t w1 = sp[1];
        if (!slot_big(w1)) {  // move the inline sessions over
            const int c1 = slot_cnt(w1), SW = a.t.words;
            for (int q = 0; q < c1; ++q) {
                const int64_t* x = sp + 2 + q * SW;
                int64_t* y = d + 2 + q * kWideWords;
                y[0] = x[0]; y[1] = x[1]; y[2] = x[2]; y[3] = SW == 4 ? x[3] : 0; y[4] = slot_fired(w1, q);
            }
            d[1] = c1;
            sp[1] = (int64_t)kBigMeta;
            due_of(a.t)[slot] = INT64_MAX;
        }
        int cnt = (int)d[1];
        if (cnt + L > a.w.ring) {
            atomicMax(&a.st->pad[1], (unsigned long long)(cnt + L));
            const unsigned long long at = atomicAdd(&a.st->overflow, 1ull);
            a.retry[at] = (uint32_t)i;
            continue;
        }
        const SessList l{d + 2, 1, kWideWords};
        for (int64_t r = i; r < j; ++r)
            if (a.slot[r] == slot) add_element<AGG>(a, l, cnt, a.w.ring, key, a.perm[r], late, merges, flags);
        d[1] = cnt;
        due_of(a.w)[g2] = wide_due(d, a.lateness);
    }
    ShardCtr& sc = a.st->sh[blockIdx.x % kShards];
    if (late) atomicAdd(&sc.late, late);
    if (merges) atomicAdd(&sc.merges, merges);
    if (flags) atomicOr(&sc.flags, flags);
    if (ins) atomicAdd(&a.st->pad[2], ins);
}

__global__ void __launch_bounds__(256) k_sess_prep(const int64_t* key, const int64_t* ts, const int64_t* val, int64_t n,
                                                   TableView t, uint32_t* slot, uint32_t* perm, int64_t* rec,
                                                   DevStatus* st) {
    unsigned long long ins = 0, flags = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the main pass's counters (nothing reads them before it)
        st->overflow = 0;
        st->pad[0] = 0;
        st->pad[1] = 0;
    }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (ts && ts[i] == INT64_MIN) flags |= GW_DF_NO_TS;
        bool inserted;
        int64_t s = find_or_insert(t, key[i], inserted);
        ins += inserted;
        if (s < 0) { flags |= GW_DF_TABLE_FULL; s = 0; }
        slot[i] = (uint32_t)s;
        perm[i] = (uint32_t)i;
        if (rec) {
            rec[2 * i] = ts[i];
            rec[2 * i + 1] = val ? val[i] : 0;
        }
    }
    block_commit(st, 0, ins, flags, 0);
}

// ---------------------------------------------------------- region-partitioned ingest
// The default session ingest.  Four launches per batch, no device-wide sort:
//  * k_sp_part: one workgroup per 4096-record tile hashes every key to its home slot and
//    writes the tile's records grouped by bucket (the top bb bits of the home slot), one run
//    per bucket, stable (arrival order inside a run); one descriptor row per tile.
//  * k_sp_transpose: descriptor rows -> one column per bucket.
//  * k_sp_group: one workgroup per bucket concatenates the bucket's runs in tile order -- the
//    bucket's records in arrival order -- and sorts them in LDS by (home slot, arrival) with a
//    stable radix sort; it writes the order and one head per home slot.
//  * k_sp_keys: one thread per home slot finds or inserts the key (the probe the sort path's
//    k_sess_prep makes, here on the line the replay needs anyway) and replays the slot's
//    records through MergingWindowSet.addWindow semantics (add_element_tv), all of the
//    batch's records of a key in arrival order.
// A key that needs the wide table (more in-flight sessions than the lane holds, or already
// wide) or finds no slot, and every key of a bucket with more than kGrpCap records, is
// punted: its records go to a punt list in arrival order, which the sort path (k_sess_prep
// ... k_sess_wide) replays after the launch.
constexpr int kSessionRegionDefault = 0;  // until it outruns the sort path on the sessions config
constexpr int kSpTile = 4096;
constexpr int kSpThreads = 1024;
constexpr int kSpWaveRecs = kSpTile / (kSpThreads / 64);  // records of one wave (a contiguous chunk)
constexpr int kSpItems = kSpWaveRecs / 64;
constexpr int kSpMaxBuckets = 1024;
constexpr size_t kSpPartLds = (size_t)kSpTile * 3 * 8 + (size_t)(kSpThreads / 64) * kSpMaxBuckets * 2;

// Pass 1.  Wave w owns the tile's records [w*256, (w+1)*256) (item it of lane l: w*256 +
// it*64 + l), so arrival order is (wave, item, lane).  Ranks within a bucket are stable:
// lanes of one bucket find each other with bb ballots, a leader per bucket bumps the wave's
// private counter, and a block scan over (bucket, wave) turns the counters into offsets.
__global__ void __launch_bounds__(kSpThreads) k_sp_part(const int64_t* key, const int64_t* ts, const int64_t* val,
                                                        int64_t n, int64_t cap, int lcap, int bb, int64_t* o_key,
                                                        longlong2* o_tv, uint32_t* row, DevStatus* st) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int64_t* s_key = reinterpret_cast<int64_t*>(smem);
    int64_t* s_ts = s_key + kSpTile;
    int64_t* s_val = s_ts + kSpTile;
    uint16_t* wcnt = reinterpret_cast<uint16_t*>(s_val + kSpTile);  // [wave][bucket]
    __shared__ uint32_t lh[kSpMaxBuckets], ls[kSpMaxBuckets];
    __shared__ uint32_t wsum[kSpThreads / 64];
    const int nb = 1 << bb, sh = lcap - bb;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t tile = blockIdx.x;
    const int64_t lo = tile * kSpTile, hi = min(n, lo + (int64_t)kSpTile);
    for (int e = tid; e < (kSpThreads / 64) * nb; e += blockDim.x) wcnt[(e / nb) * kSpMaxBuckets + e % nb] = 0;
    int64_t k[kSpItems], t[kSpItems], v[kSpItems];
#pragma unroll
    for (int it = 0; it < kSpItems; ++it) {  // all loads in flight first
        const int64_t i = lo + w * kSpWaveRecs + it * 64 + lane;
        k[it] = 0; t[it] = 0; v[it] = 0;
        if (i < hi) {
            k[it] = __builtin_nontemporal_load(key + i);
            t[it] = __builtin_nontemporal_load(ts + i);
            if (val) v[it] = __builtin_nontemporal_load(val + i);
        }
    }
    __syncthreads();
    unsigned long long flags = 0;
    uint16_t* my = wcnt + w * kSpMaxBuckets;
    uint32_t bk[kSpItems], rk[kSpItems];
#pragma unroll
    for (int it = 0; it < kSpItems; ++it) {
        const int64_t i = lo + w * kSpWaveRecs + it * 64 + lane;
        const bool ok = i < hi;
        if (ok && t[it] == INT64_MIN) flags |= GW_DF_NO_TS;
        const uint32_t b = !ok ? 0u
                           : k[it] == kEmptyKey ? (uint32_t)(nb - 1)
                                                : (uint32_t)((slot_hash(k[it]) & (uint64_t)(cap - 1)) >> sh);
        uint64_t peers = __ballot(ok);
        for (int q = 0; q < bb; ++q) {
            const uint64_t m = __ballot(ok && ((b >> q) & 1u));
            peers &= ((b >> q) & 1u) ? m : ~m;
        }
        uint32_t old = 0;
        const int leader = ok ? __ffsll((long long)peers) - 1 : 0;
        if (ok && lane == leader) {
            old = my[b];
            my[b] = (uint16_t)(old + __popcll(peers));
        }
        old = __shfl(old, leader);
        bk[it] = ok ? b : ~0u;
        rk[it] = old + (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
    }
    __syncthreads();
    {  // bucket totals, exclusive scan over buckets, then per-(wave, bucket) offsets in place
        uint32_t x = 0;
        if (tid < nb)
            for (int q = 0; q < kSpThreads / 64; ++q) x += wcnt[q * kSpMaxBuckets + tid];
        uint32_t incl = x;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t up = __shfl_up(incl, o);
            if (lane >= o) incl += up;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (int q = 0; q < w; ++q) off += wsum[q];
        if (tid < nb) {
            ls[tid] = off + incl - x;
            lh[tid] = x;
            uint32_t r = off + incl - x;
            for (int q = 0; q < kSpThreads / 64; ++q) {
                const uint32_t c = wcnt[q * kSpMaxBuckets + tid];
                wcnt[q * kSpMaxBuckets + tid] = (uint16_t)r;
                r += c;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kSpItems; ++it) {
        if (bk[it] == ~0u) continue;
        const uint32_t j = my[bk[it]] + rk[it];
        s_key[j] = k[it];
        s_ts[j] = t[it];
        s_val[j] = v[it];
    }
    __syncthreads();
    const int64_t base = tile * kSpTile;
    const int cnt = (int)(hi - lo);
    for (int j = tid; j < cnt; j += blockDim.x) {  // read back by the grouping and the replay
        o_key[base + j] = s_key[j];
        o_tv[base + j] = longlong2{s_ts[j], s_val[j]};
    }
    for (int b = tid; b < nb; b += blockDim.x) row[tile * nb + b] = (ls[b] << 16) | lh[b];
    block_commit(st, 0, 0, flags, 0);
}

// Descriptor rows [tile][bucket] -> columns [bucket][tile] (64 x 64 blocks through LDS).
__global__ void __launch_bounds__(256) k_sp_transpose(const uint32_t* row, uint32_t* col, int64_t ntiles, int nb) {
    __shared__ uint32_t tt[64][65];
    const int64_t t0 = (int64_t)blockIdx.x * 64;
    const int b0 = blockIdx.y * 64;
    for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) {
        const int tl = e >> 6, bl = e & 63;
        const int64_t t = t0 + tl;
        tt[tl][bl] = (t < ntiles && b0 + bl < nb) ? row[t * nb + b0 + bl] : 0u;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) {
        const int bl = e >> 6, tl = e & 63;
        const int64_t t = t0 + tl;
        if (t < ntiles && b0 + bl < nb) col[(int64_t)(b0 + bl) * ntiles + t] = tt[tl][bl];
    }
}

// Session words per slot: start, end, acc (+ count for averages).
template <int AGG>
__device__ __forceinline__ constexpr int sess_words() {
    return (AGG == GW_AVG_I64 || AGG == GW_AVG_F64) ? 4 : 3;
}

// Grouping (k_sp_group): one workgroup per bucket sorts the bucket's records of the batch by
// (local home slot, arrival) in LDS -- a stable two-pass radix sort over the home bits of
// 32-bit keys (home << 14 | position) -- and writes the buffer offsets in that order plus
// one head per home slot.  A bucket holds at most kGrpCap records; the records of a bucket
// with more (a hot key, a batch far above the table's design size) go to the punt list.
constexpr int kGrpCap = 16384;
constexpr int kGrpPosBits = 14;
constexpr int kGrpThreads = 1024;
constexpr int kGrpItems = kGrpCap / kGrpThreads;     // per thread per radix pass
constexpr int kGrpWaveRecs = kGrpCap / (kGrpThreads / 64);
constexpr int kGrpMaxHomeBits = 31 - kGrpPosBits - 1;  // + the sentinel's code
constexpr int kGrpBins = 512;
constexpr size_t kGrpLds = (size_t)kGrpCap * 4 * 2 + (size_t)(kGrpThreads / 64) * kGrpBins * 2;

// One stable LSD radix pass over x[0..n) -> y, digit = (v >> sh) & (2^db - 1), db <= 9.
// Wave w owns positions [w*kGrpWaveRecs, (w+1)*kGrpWaveRecs) (item it of lane l at
// w*kGrpWaveRecs + it*64 + l), so (wave, item, lane) is the input order; lanes of one digit
// find each other with db ballots, and a leader per digit bumps the wave's counter.
__device__ __forceinline__ void grp_radix_pass(const uint32_t* x, uint32_t* y, int n, int sh, int db,
                                               uint16_t* wcnt, uint32_t* wsum) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nbins = 1 << db;
    for (int e = tid; e < (kGrpThreads / 64) * kGrpBins; e += blockDim.x) wcnt[e] = 0;
    __syncthreads();
    uint16_t* my = wcnt + w * kGrpBins;
    uint32_t v[kGrpItems], rk[kGrpItems];
#pragma unroll
    for (int it = 0; it < kGrpItems; ++it) {
        const int pos = w * kGrpWaveRecs + it * 64 + lane;
        const bool ok = pos < n;
        v[it] = ok ? x[pos] : 0u;
        const uint32_t d = (v[it] >> sh) & (uint32_t)(nbins - 1);
        uint64_t peers = __ballot(ok);
        if (!peers) { rk[it] = 0; continue; }  // wave-uniform
        for (int q = 0; q < db; ++q) {
            const uint64_t m = __ballot(ok && ((d >> q) & 1u));
            peers &= ((d >> q) & 1u) ? m : ~m;
        }
        uint32_t old = 0;
        const int leader = ok ? __ffsll((long long)peers) - 1 : 0;
        if (ok && lane == leader) {
            old = my[d];
            my[d] = (uint16_t)(old + __popcll(peers));
        }
        old = __shfl(old, leader);
        rk[it] = old + (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
    }
    __syncthreads();
    {  // digit totals -> exclusive scan over digits -> per-(wave, digit) offsets in place
        const int per = kGrpBins / kGrpThreads > 0 ? kGrpBins / kGrpThreads : 1;
        (void)per;
        uint32_t tot = 0;
        if (tid < nbins)
            for (int q = 0; q < kGrpThreads / 64; ++q) tot += wcnt[q * kGrpBins + tid];
        uint32_t incl = tot;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t up = __shfl_up(incl, o);
            if (lane >= o) incl += up;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (int q = 0; q < w; ++q) off += wsum[q];
        if (tid < nbins) {
            uint32_t r = off + incl - tot;
            for (int q = 0; q < kGrpThreads / 64; ++q) {
                const uint32_t c = wcnt[q * kGrpBins + tid];
                wcnt[q * kGrpBins + tid] = (uint16_t)r;
                r += c;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < kGrpItems; ++it) {
        const int pos = w * kGrpWaveRecs + it * 64 + lane;
        if (pos < n) y[my[(v[it] >> sh) & (uint32_t)(nbins - 1)] + rk[it]] = v[it];
    }
    __syncthreads();
}

// grid: one workgroup per bucket.  Outputs per bucket b (at b * kGrpCap): perm[] the
// pass-1 buffer offsets of the bucket's records in (home, arrival) order, shd[] heads (sorted
// index | local home << 14); grp_n[2b] = records, grp_n[2b+1] = heads (both 0 for an
// oversize bucket, whose records went to the punt list).  gsrc: scratch, offset by position.
__global__ void __launch_bounds__(kGrpThreads) k_sp_group(SegArgs a, uint32_t* gsrc, uint32_t* perm, uint32_t* shd,
                                                          uint32_t* grp_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* ka = reinterpret_cast<uint32_t*>(smem);
    uint32_t* kb = ka + kGrpCap;
    uint16_t* wcnt = reinterpret_cast<uint16_t*>(kb + kGrpCap);
    __shared__ uint32_t wsum[kGrpThreads / 64];
    __shared__ uint32_t s_tot, s_nh;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t b = blockIdx.x;
    const uint32_t* col = a.col + b * a.ntiles;
    const int sh = a.lcap - a.bb;
    const uint64_t hmask = ((uint64_t)1 << sh) - 1;
    const uint32_t sent = 1u << sh;
    uint32_t* gs = gsrc + b * kGrpCap;
    // records of the bucket; an oversize bucket's records all go to the punt list (arrival
    // order), which the sort path replays: its keys are disjoint from the other buckets'
    {
        uint32_t c = 0;
        for (int64_t t = tid; t < a.ntiles; t += blockDim.x) c += col[t] & 0xffffu;
        c = (uint32_t)wave_sum(c);
        if (lane == 0) wsum[w] = c;
        __syncthreads();
        if (tid == 0) {
            uint32_t tot = 0;
            for (int q = 0; q < kGrpThreads / 64; ++q) tot += wsum[q];
            s_tot = tot;
            s_nh = tot > (uint32_t)kGrpCap ? (uint32_t)atomicAdd(&a.st->overflow, (unsigned long long)tot) : 0u;
        }
        __syncthreads();
    }
    const uint32_t n = s_tot;
    const bool over = n > (uint32_t)kGrpCap;
    const uint32_t pbase = s_nh;
    // the bucket's runs in tile order (arrival order): thread t takes tiles [3t, 3t + 3) of each
    // chunk of 3 * kGrpThreads tiles, 8 records at a time with their loads issued together
    uint32_t running = 0;
    for (int64_t c0 = 0; c0 < a.ntiles; c0 += 3 * kGrpThreads) {
        uint32_t d[3], sum = 0;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int64_t t = c0 + 3 * tid + q;
            d[q] = t < a.ntiles ? col[t] : 0u;
            sum += d[q] & 0xffffu;
        }
        uint32_t incl = sum;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t up = __shfl_up(incl, o);
            if (lane >= o) incl += up;
        }
        if (lane == 63) wsum[w] = incl;
        __syncthreads();
        uint32_t pre = running + incl - sum, tot = 0;
        for (int q = 0; q < kGrpThreads / 64; ++q) {
            if (q < w) pre += wsum[q];
            tot += wsum[q];
        }
        const uint32_t c0n = d[0] & 0xffffu, c1n = d[1] & 0xffffu;
        uint32_t s3[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) s3[q] = (uint32_t)((c0 + 3 * tid + q) * kSpTile + (d[q] >> 16));
        for (uint32_t u0 = 0; u0 < sum; u0 += 8) {
            uint32_t sv[8];
            int64_t kk[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t uu = u0 + u;
                sv[u] = uu < c0n ? s3[0] + uu : uu < c0n + c1n ? s3[1] + (uu - c0n) : s3[2] + (uu - c0n - c1n);
                kk[u] = uu < sum ? a.p_key[sv[u]] : 0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t uu = u0 + u;
                if (uu >= sum) break;
                const uint32_t pos = pre + uu;
                if (over) {
                    const longlong2 tv = a.p_tv[sv[u]];
                    a.pu_key[pbase + pos] = kk[u];
                    a.pu_ts[pbase + pos] = tv.x;
                    a.pu_val[pbase + pos] = tv.y;
                } else {
                    const uint32_t lh = kk[u] == kEmptyKey ? sent : (uint32_t)(slot_hash(kk[u]) & hmask);
                    ka[pos] = (lh << kGrpPosBits) | pos;
                    gs[pos] = sv[u];
                }
            }
        }
        running += tot;
        __syncthreads();  // wsum is rewritten by the next chunk
    }
    if (over) {
        if (tid == 0) { grp_n[2 * b] = 0; grp_n[2 * b + 1] = 0; }
        return;
    }
    // home bits [kGrpPosBits, kGrpPosBits + sh + 1): two passes
    const int hb = sh + 1, db0 = (hb + 1) / 2, db1 = hb - db0;
    grp_radix_pass(ka, kb, (int)n, kGrpPosBits, db0, wcnt, wsum);
    const uint32_t* fin = kb;
    if (db1 > 0) {
        grp_radix_pass(kb, ka, (int)n, kGrpPosBits + db0, db1, wcnt, wsum);
        fin = ka;
    }
    uint32_t* po = perm + b * kGrpCap;
    uint32_t* ho = shd + b * kGrpCap;
    uint32_t nh = 0;  // heads in sorted order: ordered compaction per chunk (waves, then lanes)
    for (uint32_t i0 = 0; i0 < n; i0 += blockDim.x) {
        const uint32_t i = i0 + tid;
        bool h = false;
        uint32_t x = 0;
        if (i < n) {
            x = fin[i];
            po[i] = gs[x & ((1u << kGrpPosBits) - 1u)];
            h = i == 0 || (fin[i - 1] >> kGrpPosBits) != (x >> kGrpPosBits);
        }
        const uint64_t bal = __ballot(h);
        if (lane == 0) wsum[w] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t base = nh, tot = 0;
        for (int q = 0; q < kGrpThreads / 64; ++q) {
            if (q < w) base += wsum[q];
            tot += wsum[q];
        }
        if (h) ho[base + __popcll(bal & ((1ull << lane) - 1ull))] = i | ((x >> kGrpPosBits) << kGrpPosBits);
        nh += tot;
        __syncthreads();  // wsum is rewritten by the next chunk
    }
    if (tid == 0) { grp_n[2 * b] = n; grp_n[2 * b + 1] = nh; }
}

// The key's list after a replay (cnt sessions in the lane) -> its slot, or to the migration
// list when it outgrew the slot (the key's later records of the batch then punt until the
// migration).
template <int AGG>
__device__ __forceinline__ void sp_store(const SegArgs& a, const SessList& l, int cnt, int64_t slot, int64_t* sp,
                                         int64_t w1) {
    constexpr int SW = sess_words<AGG>();
    if (cnt <= a.t.ring) {
        uint64_t fired = 0;
        int64_t due = INT64_MAX;
        for (int q = 0; q < cnt; ++q) {
            const Sess v = sl_get(l, q);
            int64_t* x = sp + 2 + q * SW;
            x[0] = v.s; x[1] = v.e; x[2] = v.a0;
            if (SW == 4) x[3] = v.a1;
            fired |= (uint64_t)(v.f != 0) << q;
            due = min(due, due_time(v.e, v.f != 0, a.lateness));
        }
        sp[1] = (int64_t)((fired << 32) | (uint64_t)(uint32_t)cnt);
        due_of(a.t)[slot] = due;
    } else {
        const unsigned long long at = atomicAdd(&a.st->pad[0], 1ull);
        int64_t* m = a.mig + at * (2 + kWideWords * kLaneSess);
        m[0] = slot;
        m[1] = cnt;
        for (int q = 0; q < cnt; ++q) {
            const Sess v = sl_get(l, q);
            int64_t* x = m + 2 + q * kWideWords;
            x[0] = v.s; x[1] = v.e; x[2] = v.a0; x[3] = v.a1; x[4] = v.f;
        }
        atomicMax(&a.st->pad[1], (unsigned long long)cnt);
        sp[1] = (int64_t)((uint64_t)w1 | kPuntMeta);
    }
}

// One key's records among the home slot's run [r0, f) of the sorted order (pr: pass-1
// offsets; r0 holds one of them, the others are the run's records with this key), in
// arrival order, against the key's slot -- seg_slot's replay, with the punt list instead of
// the wide pass.
template <int AGG>
__device__ __forceinline__ void sp_key(const SegArgs& a, const SessList& l, int64_t key, uint32_t r0, uint32_t f,
                                       const uint32_t* pr, unsigned long long& late, unsigned long long& merges,
                                       unsigned long long& flags, unsigned long long& ins) {
    constexpr int SW = sess_words<AGG>();
    int64_t L = 0;
    for (uint32_t q = r0; q < f; ++q) L += a.p_key[pr[q]] == key;
    bool inserted;
    const int64_t slot = find_or_insert(a.t, key, inserted);
    int64_t* sp = slot >= 0 ? slot_ptr(a.t, slot) : nullptr;
    if (sp) ins += inserted;
    const int64_t w1 = sp ? sp[1] : 0;
    bool ok = sp && !((uint64_t)w1 & (kBigMeta | kPuntMeta));
    bool dry = ok && slot_cnt(w1) + L > kLaneSess;  // could outgrow the lane
    const bool effects = a.lateness > 0 || a.lo_key;
    const unsigned long long l0 = late, m0 = merges;
    int cnt = 0;
    while (ok) {  // at most two replays: dry, then (with effects) the real one
        cnt = slot_cnt(w1);
        for (int q = 0; q < cnt; ++q) {
            const int64_t* x = sp + 2 + q * SW;
            sl_put(l, q, Sess{x[0], x[1], x[2], SW == 4 ? x[3] : 0, (int64_t)slot_fired(w1, q)});
        }
        for (uint32_t q = r0; q < f && ok; ++q) {
            const uint32_t o = pr[q];
            if (a.p_key[o] != key) continue;
            const longlong2 tv = a.p_tv[o];
            ok = add_element_tv<AGG>(a, l, cnt, kLaneSess, key, tv.x, tv.y, late, merges, flags, dry);
        }
        if (!ok || !dry || !effects) break;
        dry = false;
        late = l0;
        merges = m0;
    }
    if (!ok) {  // punt the key's records of the batch (kPuntMeta: also any that come after)
        late = l0;
        merges = m0;
        unsigned long long at = atomicAdd(&a.st->overflow, (unsigned long long)L);
        for (uint32_t q = r0; q < f; ++q) {
            const uint32_t o = pr[q];
            if (a.p_key[o] != key) continue;
            const longlong2 tv = a.p_tv[o];
            a.pu_key[at] = key;
            a.pu_ts[at] = tv.x;
            a.pu_val[at] = tv.y;
            ++at;
        }
        if (sp) sp[1] = (int64_t)((uint64_t)w1 | kPuntMeta);
        return;
    }
    sp_store<AGG>(a, l, cnt, slot, sp, w1);
}

// Every key of a home slot's run [e, f), in order of its first record (several keys per home
// slot are rare), through sp_key.
template <int AGG>
__device__ __forceinline__ void sp_run(const SegArgs& a, const SessList& l, uint32_t e, uint32_t f, const uint32_t* pr,
                                       unsigned long long& late, unsigned long long& merges,
                                       unsigned long long& flags, unsigned long long& ins) {
    for (uint32_t r = e; r < f;) {
        sp_key<AGG>(a, l, a.p_key[pr[r]], r, f, pr, late, merges, flags, ins);
        uint32_t nx = f;
        for (uint32_t q = r + 1; q < f && nx == f; ++q) {
            const int64_t kq = a.p_key[pr[q]];
            bool seen = false;
            for (uint32_t z = e; z < q && !seen; ++z) seen = a.p_key[pr[z]] == kq;
            if (!seen) nx = q;
        }
        r = nx;
    }
}

// Replay: one thread per home slot.  A persistent grid (a multiple of 8 workgroups): the
// workgroups with blockIdx % 8 == x walk the buckets b == x (mod 8) and deal their chunks of
// 256 heads round-robin among themselves -- under the round-robin placement of
// workgroups on the 8 XCDs (speed only, never correctness) a bucket's pass-1 lines are read
// into one L2 and its records gathered from there.  The thread loads its home slot's line
// with the offsets of its first kSpFast records, then their keys and (timestamp, value)
// pairs.  A run of one key that finds its slot within kSpProbe lines of the home slot (or
// claims a free one there) replays from registers, kSpFast records at a time; the rest go on
// the slow list for k_sp_slow (longer probes, several keys per home slot, the wide table, a
// list that could outgrow the lane under allowed lateness or the side output).
constexpr int kSpKeyThreads = 256;
constexpr int kSpFast = 4;
constexpr int kSpProbe = 4;
template <int AGG>
__global__ void __launch_bounds__(kSpKeyThreads) k_sp_keys(SegArgs a, const uint32_t* perm, const uint32_t* shd,
                                                           const uint32_t* grp_n, int nb) {
    constexpr int SW = sess_words<AGG>();
    constexpr uint32_t pm = (1u << kGrpPosBits) - 1u;
    __shared__ int64_t lane[5 * kLaneSess * kSpKeyThreads];
    const SessList l{lane + threadIdx.x, kLaneSess * kSpKeyThreads, kSpKeyThreads};
    const int sh = a.lcap - a.bb;
    const uint32_t sent = 1u << sh;
    const bool effects = a.lateness > 0 || a.lo_key;
    const int xg = blockIdx.x & 7, per = gridDim.x >> 3, me = blockIdx.x >> 3;
    unsigned long long late = 0, merges = 0, flags = 0, ins = 0;
    uint32_t base = 0;  // chunks of this XCD group's earlier buckets: chunk g goes to workgroup g % per
    for (int64_t b = xg; b < nb; b += 8) {
        const uint32_t n = grp_n[2 * b], nh = grp_n[2 * b + 1];
        const uint32_t* pr = perm + b * kGrpCap;
        const uint32_t* hd = shd + b * kGrpCap;
        const uint32_t nch = (nh + kSpKeyThreads - 1) / kSpKeyThreads;
        const uint32_t c0 = (uint32_t)((me - (int)(base % (uint32_t)per) + per) % per);
        base += nch;
        for (uint32_t c = c0; c < nch; c += per) {
            const uint32_t j = c * kSpKeyThreads + threadIdx.x;
            if (j >= nh) continue;
            const uint32_t h = hd[j];
            const uint32_t e = h & pm, lh = h >> kGrpPosBits;
            const uint32_t f = j + 1 < nh ? (hd[j + 1] & pm) : n;
            const uint32_t L = f - e;
            const bool sentinel = lh == sent;
            int64_t slot = sentinel ? a.t.cap : ((b << sh) | (int64_t)lh);
            int64_t cur[8], rk[kSpFast], rt[kSpFast], rv[kSpFast];
            uint32_t ro[kSpFast];
// (macros, not lambdas: a lambda capturing these arrays by reference would put them in scratch)
#define SP_LOAD_LINE(sl)                                                                   \
    do {                                                                                   \
        const longlong2* p_ = reinterpret_cast<const longlong2*>(slot_ptr(a.t, (sl)));     \
        _Pragma("unroll") for (int x_ = 0; x_ < 4; ++x_) {                                 \
            const longlong2 y_ = p_[x_];                                                   \
            cur[2 * x_] = y_.x;                                                            \
            cur[2 * x_ + 1] = y_.y;                                                        \
        }                                                                                  \
    } while (0)
#define SP_LOAD_OFFS(c)  /* pass-1 offsets of records [c, c + kSpFast) of the run (clamped) */ \
    do {                                                                                   \
        _Pragma("unroll") for (int u_ = 0; u_ < kSpFast; ++u_) ro[u_] = pr[(c) + u_ < f ? (c) + u_ : e]; \
    } while (0)
#define SP_LOAD_RECS()                                                                     \
    do {                                                                                   \
        _Pragma("unroll") for (int u_ = 0; u_ < kSpFast; ++u_) {                           \
            rk[u_] = a.p_key[ro[u_]];                                                      \
            const longlong2 tv_ = a.p_tv[ro[u_]];                                          \
            rt[u_] = tv_.x;                                                                \
            rv[u_] = tv_.y;                                                                \
        }                                                                                  \
    } while (0)
            SP_LOAD_LINE(slot);
            SP_LOAD_OFFS(e);
            SP_LOAD_RECS();
            // the run's keys: one, or two (home slots shared by two keys of the batch) in a run
            // of at most kSpFast records; anything else goes to k_sp_slow
            const int64_t k0 = rk[0];
            int64_t k1 = k0;
            bool fit = true;
            uint32_t L0 = L;
            if (L <= (uint32_t)kSpFast) {
                L0 = 1;
#pragma unroll
                for (int u = 1; u < kSpFast; ++u) {
                    if ((uint32_t)u >= L) continue;
                    if (rk[u] == k0) { ++L0; continue; }
                    if (k1 == k0) k1 = rk[u];
                    else if (rk[u] != k1) fit = false;
                }
            } else {
                for (uint32_t q = e;;) {
#pragma unroll
                    for (int u = 1; u < kSpFast; ++u) fit = fit && (q + u >= f || rk[u] == k0);
                    q += kSpFast;
                    if (q >= f || !fit) break;
                    SP_LOAD_OFFS(q);
                    SP_LOAD_RECS();
                    fit = fit && rk[0] == k0;
                }
                SP_LOAD_OFFS(e);
                SP_LOAD_RECS();
            }
            const bool two = k1 != k0;
            const uint32_t L1 = L - L0;
            // each key's slot: its home slot's line, or up to kSpProbe - 1 lines further
            // (a free slot is claimed -- harmless if the run then goes to k_sp_slow after all)
            int64_t slot0 = slot, slot1 = slot, c1w[8];
#define SP_PROBE(KEY, SL, FOUND)                                                                           \
    do {                                                                                                   \
        for (int pr_ = 0; pr_ < kSpProbe && !(FOUND); ++pr_) {                                             \
            if (cur[0] == (KEY)) { FOUND = true; break; }                                                  \
            if (cur[0] == kEmptyKey) {                                                                     \
                const unsigned long long prev_ = atomicCAS((unsigned long long*)slot_ptr(a.t, SL),         \
                                                           (unsigned long long)kEmptyKey, (unsigned long long)(KEY)); \
                if (prev_ == (unsigned long long)kEmptyKey) { /* new key: a free slot has word 1 == 0 */   \
                    FOUND = true;                                                                          \
                    ins++;                                                                                 \
                    cur[1] = 0;                                                                            \
                    break;                                                                                 \
                }                                                                                          \
            }                                                                                              \
            SL = (SL + 1) & (a.t.cap - 1);                                                                 \
            SP_LOAD_LINE(SL);                                                                              \
        }                                                                                                  \
    } while (0)
            bool f0 = sentinel, f1 = true;
            if (fit) SP_PROBE(k0, slot0, f0);
            if (fit && two && f0) {
#pragma unroll
                for (int x = 0; x < 8; ++x) c1w[x] = cur[x];  // key 0's line
                f1 = false;
                SP_LOAD_LINE(slot1);
                SP_PROBE(k1, slot1, f1);
#pragma unroll
                for (int x = 0; x < 8; ++x) {  // cur: key 0's line again, c1w: key 1's
                    const int64_t t = cur[x];
                    cur[x] = c1w[x];
                    c1w[x] = t;
                }
            }
#undef SP_PROBE
            const int64_t w10 = cur[1], w11 = two ? c1w[1] : 0;
            const bool fast = fit && f0 && f1 && !((uint64_t)(w10 | w11) & (kBigMeta | kPuntMeta)) &&
                              (!effects || (slot_cnt(w10) + L0 <= kLaneSess && slot_cnt(w11) + L1 <= kLaneSess));
            if (fast) {  // each key's records replay from registers against its loaded line
#pragma unroll 1
                for (int ki = 0; ki < (two ? 2 : 1); ++ki) {
                    const int64_t key = ki ? k1 : k0;
                    const int64_t sl = ki ? slot1 : slot0;
                    if (ki) {
#pragma unroll
                        for (int x = 0; x < 8; ++x) cur[x] = c1w[x];
                    }
                    const int64_t w1 = cur[1];
                    int64_t* sp = slot_ptr(a.t, sl);
                    int cnt = slot_cnt(w1);
#pragma unroll
                    for (int q = 0; q < (8 - 2) / SW; ++q)
                        if (q < cnt)
                            sl_put(l, q, Sess{cur[2 + q * SW], cur[3 + q * SW], cur[4 + q * SW],
                                              SW == 4 ? cur[5 + q * SW] : 0, (int64_t)slot_fired(w1, q)});
                    const unsigned long long l0 = late, m0 = merges;
                    bool ok = true;
                    for (uint32_t q = e; q < f && ok; q += kSpFast) {
                        if (q != e) {
                            SP_LOAD_OFFS(q);
                            SP_LOAD_RECS();
                        }
                        const int m = (int)min((uint32_t)kSpFast, f - q);
                        for (int u = 0; u < m && ok; ++u) {
                            int64_t t = rt[0], v = rv[0], kk = rk[0];  // record u by selects: no scratch
#pragma unroll
                            for (int x = 1; x < kSpFast; ++x) {
                                t = u == x ? rt[x] : t;
                                v = u == x ? rv[x] : v;
                                kk = u == x ? rk[x] : kk;
                            }
                            if (kk == key)
                                ok = add_element_tv<AGG>(a, l, cnt, kLaneSess, key, t, v, late, merges, flags, false);
                        }
                    }
                    if (ok) {
                        sp_store<AGG>(a, l, cnt, sl, sp, w1);
                    } else {  // outgrew the lane (no effects were written): punt the key's records
                        late = l0;
                        merges = m0;
                        const uint32_t Lk = ki ? L1 : L0;
                        unsigned long long at = atomicAdd(&a.st->overflow, (unsigned long long)Lk);
                        for (uint32_t q = e; q < f; ++q) {
                            const uint32_t o = pr[q];
                            if (a.p_key[o] != key) continue;
                            const longlong2 tv = a.p_tv[o];
                            a.pu_key[at] = key;
                            a.pu_ts[at] = tv.x;
                            a.pu_val[at] = tv.y;
                            ++at;
                        }
                        sp[1] = (int64_t)((uint64_t)w1 | kPuntMeta);
                    }
                    if (!ki && two) {  // key 1's records: reload the first chunk (the loop moved on)
                        SP_LOAD_OFFS(e);
                        SP_LOAD_RECS();
                    }
                }
            } else {  // k_sp_slow replays it (a dense launch: no divergence against the fast runs)
                if (a.exp) {  // GW_SP_EXP: why (two shards' spare counters)
                    if (!fit) atomicAdd(&a.st->sh[0].pad0, 1ull);
                    else if (!(f0 && f1)) atomicAdd(&a.st->sh[0].pad1, 1ull);
                    else if ((uint64_t)(w10 | w11) & (kBigMeta | kPuntMeta)) atomicAdd(&a.st->sh[1].pad0, 1ull);
                    else atomicAdd(&a.st->sh[1].pad1, 1ull);
                }
                const uint64_t bal = __ballot(true);
                unsigned long long at = 0;
                const int ld = __ffsll((long long)bal) - 1;
                if (__lane_id() == ld) at = atomicAdd(&a.st->spills, (unsigned long long)__popcll(bal));
                at = __shfl(at, ld);
                a.slow[at + __popcll(bal & ((1ull << __lane_id()) - 1ull))] = ((uint32_t)b << kGrpPosBits) | j;
            }
#undef SP_LOAD_LINE
#undef SP_LOAD_OFFS
#undef SP_LOAD_RECS
        }
    }
    block_commit(a.st, late, ins, flags, 0, 0, merges);
}

// The home slots k_sp_keys left (a.slow, st->spills of them) through sp_run.
template <int AGG>
__global__ void __launch_bounds__(kSpKeyThreads) k_sp_slow(SegArgs a, const uint32_t* perm, const uint32_t* shd,
                                                           const uint32_t* grp_n) {
    constexpr uint32_t pm = (1u << kGrpPosBits) - 1u;
    __shared__ int64_t lane[5 * kLaneSess * kSpKeyThreads];
    const SessList l{lane + threadIdx.x, kLaneSess * kSpKeyThreads, kSpKeyThreads};
    const uint64_t ns = a.st->spills;
    unsigned long long late = 0, merges = 0, flags = 0, ins = 0;
    for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < ns; x += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t id = a.slow[x];
        const int64_t b = id >> kGrpPosBits;
        const uint32_t j = id & pm;
        const uint32_t n = grp_n[2 * b], nh = grp_n[2 * b + 1];
        const uint32_t e = shd[b * kGrpCap + j] & pm;
        const uint32_t f = j + 1 < nh ? (shd[b * kGrpCap + j + 1] & pm) : n;
        sp_run<AGG>(a, l, e, f, perm + b * kGrpCap, late, merges, flags, ins);
    }
    block_commit(a.st, late, ins, flags, 0, 0, merges);
}

// After a replay with punts: clear the punt marks before the sort path replays the list.
__global__ void __launch_bounds__(256) k_sp_unpunt(TableView t, const int64_t* pk, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t slot = find_slot(t, pk[i]);
        if (slot < 0) continue;
        int64_t* sp = slot_ptr(t, slot);
        if ((uint64_t)sp[1] & kPuntMeta) atomicAnd((unsigned long long*)(sp + 1), ~(unsigned long long)kPuntMeta);
    }
}

// Fire sweep, part 1: stream the due array (8 B per slot) and list the slots with
// something due at `wm` -- a small fraction: the sessions that close at this watermark.
// Each workgroup scans one contiguous chunk with 16-B loads (4 per lane in flight),
// collects its hits in LDS and reserves list space with one atomic at the end.
constexpr int kDueBuf = 4096;
__global__ void __launch_bounds__(256) k_sess_due_scan(TableView t, int64_t wm, uint32_t* list, DevStatus* st) {
    __shared__ uint32_t buf[kDueBuf];
    __shared__ unsigned cnt;
    __shared__ unsigned long long gbase;
    const int64_t nslots = t.cap + 1;
    const int64_t* due = due_of(t);
    constexpr int kStep = 256 * 2 * 4;  // slots per workgroup iteration
    const int64_t chunk = ((nslots + gridDim.x - 1) / gridDim.x + kStep - 1) / kStep * kStep;
    const int64_t lo = blockIdx.x * chunk, hi = min(nslots, lo + chunk);
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    auto hit = [&](int64_t i) {
        const unsigned p = atomicAdd(&cnt, 1u);
        if (p < kDueBuf) {
            buf[p] = (uint32_t)i;
        } else {  // a watermark that makes most slots due: straight to the list
            list[atomicAdd(&st->n_refire, 1ull)] = (uint32_t)i;
        }
    };
    for (int64_t b = lo; b < hi; b += kStep) {
        int64_t d[8];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = b + u * 512 + 2 * threadIdx.x;
            if (i + 1 < hi) {
                const longlong2 x = *reinterpret_cast<const longlong2*>(due + i);
                d[2 * u] = x.x;
                d[2 * u + 1] = x.y;
            } else {
                d[2 * u] = i < hi ? due[i] : INT64_MAX;
                d[2 * u + 1] = INT64_MAX;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = b + u * 512 + 2 * threadIdx.x;
            if (d[2 * u] <= wm && i < hi) hit(i);
            if (d[2 * u + 1] <= wm && i + 1 < hi) hit(i + 1);
        }
    }
    __syncthreads();
    const unsigned c = min(cnt, (unsigned)kDueBuf);
    if (threadIdx.x == 0 && c) gbase = atomicAdd(&st->n_refire, (unsigned long long)c);
    __syncthreads();
    for (unsigned j = threadIdx.x; j < c; j += blockDim.x) list[gbase + j] = buf[j];
}

// Part 2: one thread per listed slot fires its due sessions (a prefix: sorted, disjoint),
// emits (key, start, end, result), drops the cleaned prefix (WindowOperator.onEventTime
// :450-494 / clearAllState :560-571), and recomputes the slot's due time.  Rows are staged
// in LDS, one row per thread per round, and flushed in bulk.
template <int AGG>
__global__ void __launch_bounds__(256) k_sess_fire(TableView t, const uint32_t* list, int64_t wm, int64_t lateness,
                                                   int purge, int64_t* o_key, int64_t* o_start, int64_t* o_end,
                                                   int64_t* o_res, DevStatus* st) {
    __shared__ RowStage rs;
    __shared__ int s_max;
    const int64_t nl = (int64_t)st->n_refire;
    const int SW = t.words;
    if (threadIdx.x == 0) rs.cnt = 0;
    __syncthreads();
    for (int64_t base = blockIdx.x * (int64_t)blockDim.x; base < nl; base += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x_i = base + threadIdx.x;
        int64_t* s = nullptr;
        int64_t i = 0;
        int cnt = 0, nf = 0, nc = 0;
        int64_t w1 = 0;
        if (x_i < nl) {
            i = list[x_i];
            s = slot_ptr(t, i);
            w1 = s[1];
            cnt = slot_big(w1) ? 0 : slot_cnt(w1);  // wide keys: k_sess_fire_wide
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
            due_of(t)[i] = inline_due(s, SW, lateness);
        }
    }
    stage_flush(rs, &st->rows, o_key, o_start, o_end, o_res);
}

// The same for the wide table (one thread per wide slot; few keys).
template <int AGG>
__global__ void __launch_bounds__(256) k_sess_fire_wide(TableView w, int64_t wm, int64_t lateness, int purge,
                                                        int64_t* o_key, int64_t* o_start, int64_t* o_end,
                                                        int64_t* o_res, DevStatus* st) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= w.cap; i += (int64_t)gridDim.x * blockDim.x) {
        if (due_of(w)[i] > wm) continue;
        int64_t* s = slot_ptr(w, i);
        const int cnt = (int)s[1];
        if (cnt <= 0) continue;
        int nf = 0, nc = 0;
        while (nf < cnt && s[2 + nf * kWideWords + 1] - 1 <= wm) ++nf;
        nc = nf;
        if (lateness > 0) {
            nc = 0;
            while (nc < nf && cleaned_at(s[2 + nc * kWideWords + 1], lateness, wm)) ++nc;
        }
        const int64_t key = i == w.cap ? kEmptyKey : s[0];
        for (int q = 0; q < nf; ++q) {
            int64_t* x = s + 2 + q * kWideWords;
            if (x[4]) continue;
            const unsigned long long o = atomicAdd(&st->rows, 1ull);
            o_key[o] = key; o_start[o] = x[0]; o_end[o] = x[1]; o_res[o] = cell_result(AGG, x[2], x[3]);
            x[4] = 1;
            if (purge) purge_acc<AGG>(x[2], x[3]);
        }
        if (nc) {
            for (int q = nc; q < cnt; ++q)
                for (int f = 0; f < kWideWords; ++f) s[2 + (q - nc) * kWideWords + f] = s[2 + q * kWideWords + f];
            s[1] = cnt - nc;
        }
        due_of(w)[i] = wide_due(s, lateness);
    }
}

// Re-hash slots holding state into a fresh table (dead keys dropped): main table (word 1 =
// count | fired bits | kBigMeta), wide table (word 1 = count), count windows (word 1 =
// element count).
__global__ void __launch_bounds__(256) k_sess_rehash(TableView o, TableView n, int words_per_slot, DevStatus* st,
                                                     int ins_field) {
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
        d[1] = s[1];
        const int nw = words_per_slot < 0 ? (int)s[1] * o.words : words_per_slot;
        for (int w = 0; w < nw; ++w) d[2 + w] = s[2 + w];
        due_of(n)[j] = due_of(o)[i];
    }
    ins = wave_sum(ins);
    flags = wave_ior(flags);
    if (__lane_id() == 0) {
        if (flags) atomicOr(&st->sh[blockIdx.x % kShards].flags, flags);
        if (ins) {
            if (ins_field < 0) atomicAdd(&st->pad[2], ins);
            else atomicAdd(&st->sh[blockIdx.x % kShards].ins, ins);
        }
    }
}

__global__ void __launch_bounds__(256) k_sess_init(TableView t) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= t.cap; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t* s = slot_ptr(t, i);
        s[0] = kEmptyKey;
        s[1] = 0;
        due_of(t)[i] = INT64_MAX;
    }
}

// Restore (gw_restore of a session snapshot): one thread per restored key.  A key with at
// most K1 restored sessions goes inline into its main slot; a key with more goes to the
// wide table (its main slot marked).  A key that already holds sessions here is counted in
// st->overflow and left untouched (blobs of one key group are never restored twice).
__global__ void __launch_bounds__(256) k_sess_restore(TableView t, TableView w, const int64_t* rk, const int64_t* roff,
                                                      const int64_t* rs, int64_t n, int64_t lateness, DevStatus* st) {
    unsigned long long ins = 0, flags = 0, ins2 = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool inserted;
        const int64_t slot = find_or_insert(t, rk[i], inserted);
        ins += inserted;
        if (slot < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        int64_t* sp = slot_ptr(t, slot);
        if (sp[1] != 0) { atomicAdd(&st->overflow, 1ull); continue; }
        const int64_t r0 = roff[i], cnt = roff[i + 1] - r0;
        if (cnt <= t.ring) {
            const int SW = t.words;
            uint64_t fired = 0;
            for (int q = 0; q < cnt; ++q) {
                const int64_t* x = rs + (r0 + q) * 5;
                int64_t* y = sp + 2 + q * SW;
                y[0] = x[0]; y[1] = x[1]; y[2] = x[2];
                if (SW == 4) y[3] = x[3];
                fired |= (uint64_t)(x[4] != 0) << q;
            }
            sp[1] = (int64_t)((fired << 32) | (uint64_t)cnt);
            due_of(t)[slot] = inline_due(sp, SW, lateness);
        } else {
            const int64_t g2 = find_or_insert(w, rk[i], inserted);
            if (g2 < 0) { flags |= GW_DF_TABLE_FULL; continue; }
            ins2 += inserted;
            int64_t* d = slot_ptr(w, g2);
            if (d[1] != 0) { atomicAdd(&st->overflow, 1ull); continue; }
            for (int64_t x = 0; x < cnt * kWideWords; ++x) d[2 + x] = rs[r0 * 5 + x];
            d[1] = cnt;
            due_of(w)[g2] = wide_due(d, lateness);
            sp[1] = (int64_t)kBigMeta;
            due_of(t)[slot] = INT64_MAX;
        }
    }
    block_commit(st, 0, ins, flags, 0);
    ins2 = wave_sum(ins2);
    if (__lane_id() == 0 && ins2) atomicAdd(&st->pad[2], ins2);
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
// with the stable radix sort (arrival order kept inside a key).  A key's run is folded in
// order by one thread; a hot key's long run (WindowWordCount's frequent words) across the
// GPU: one thread or wave per pane folds the pane's elements, then one thread per firing
// folds the window's n panes.
struct CountGeom {
    int64_t size, slide, g;
};
constexpr int kCntLongRun = 16;    // longer runs are spread over panes and firings

template <int AGG>
__device__ __forceinline__ void cnt_emit(DevStatus* st, int64_t* ok, int64_t* os, int64_t* oe, int64_t* orr, int64_t key,
                                         int64_t c, int64_t len, int64_t r0, int64_t r1) {
    const unsigned long long o = atomicAdd(&st->rows, 1ull);
    ok[o] = key;
    os[o] = c - len;
    oe[o] = c;
    orr[o] = cell_result(AGG, r0, r1);
}

template <int AGG>
__global__ void __launch_bounds__(256) k_cnt_apply(TableView t, CountGeom G, const uint32_t* ks, const uint32_t* perm,
                                                   int64_t n, const int64_t* val, int64_t* ok, int64_t* os,
                                                   int64_t* oe, int64_t* orr, uint32_t* longs, DevStatus* st) {
    constexpr int W = (AGG == GW_AVG_I64 || AGG == GW_AVG_F64) ? 2 : 1;
    const int R = t.ring;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t slot = ks[i];
        if (i > 0 && ks[i - 1] == slot) continue;  // not the head of a key's run
        int64_t j = i + 1;
        while (j < n && ks[j] == slot && j - i <= kCntLongRun) ++j;
        if (j - i > kCntLongRun) {  // a hot key: k_cnt_long
            const unsigned long long at = atomicAdd(&st->overflow, 1ull);
            longs[at] = (uint32_t)i;
            continue;
        }
        int64_t* sp = slot_ptr(t, (int64_t)slot);
        int64_t* cells = sp + 2;
        const int64_t key = sp[0];  // the sentinel slot's key word is Long.MIN_VALUE, its key
        int64_t c = sp[1];
        for (int64_t r = i; r < j; ++r) {
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
                cnt_emit<AGG>(st, ok, os, oe, orr, key, c, len, r0, r1);
            }
        }
        sp[1] = c;
    }
}

// Hot keys' long runs: spread over the whole GPU in three launches.  A plan row per run
// (arrival start i, length L, element count c0 before the batch, slot) and exclusive
// prefix sums of its panes [c0/g, (c0+L-1)/g] and firings (counts c = f*slide in
// (c0, c0+L]) give every pane and every firing a global index:
//   k_cnt_panes  one thread (g < 16) or one wave per pane folds the pane's elements (the
//                first pane starts from its ring cell when it began before the batch);
//   k_cnt_fires  one thread per firing folds its n panes from the pane values or, for
//                panes before the batch, the key's ring;
//   k_cnt_ring   the run's last n panes go back to the ring, the count to the slot.
enum { kPlanI, kPlanL, kPlanC0, kPlanSlot, kPlanWords = 4 };

__global__ void __launch_bounds__(256) k_cnt_long_info(TableView t, CountGeom G, const uint32_t* ks, int64_t n,
                                                       const uint32_t* longs, int64_t nl, int64_t* plan,
                                                       int64_t* poff, int64_t* foff) {
    const int64_t l = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (l >= nl) return;
    const int64_t i = longs[l];
    const uint32_t slot = ks[i];
    int64_t lo = i + 1, hi = n;  // ks is sorted: the run ends at the first other slot
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (ks[mid] == slot) lo = mid + 1; else hi = mid;
    }
    int64_t* p = plan + l * kPlanWords;
    p[kPlanI] = i;
    p[kPlanL] = lo - i;
    const int64_t c0 = slot_ptr(t, (int64_t)slot)[1], L = lo - i;
    p[kPlanC0] = c0;
    p[kPlanSlot] = slot;
    poff[l] = (c0 + L - 1) / G.g - c0 / G.g + 1;  // panes and firings of the run (scanned next)
    foff[l] = (c0 + L) / G.slide - c0 / G.slide;
}

// Exclusive prefix sums of the runs' pane and firing counts, in place (one workgroup;
// off[nl] = the total).
__global__ void __launch_bounds__(1024) k_cnt_plan_scan(int64_t* poff, int64_t* foff, int64_t nl) {
    __shared__ int64_t sp[1024], sf[1024];
    const int64_t per = (nl + 1023) / 1024;
    const int64_t b = threadIdx.x * per, e = min(nl, b + per);
    int64_t tp = 0, tf = 0;
    for (int64_t x = b; x < e; ++x) { tp += poff[x]; tf += foff[x]; }
    sp[threadIdx.x] = tp;
    sf[threadIdx.x] = tf;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
        const int64_t ap = threadIdx.x >= o ? sp[threadIdx.x - o] : 0, af = threadIdx.x >= o ? sf[threadIdx.x - o] : 0;
        __syncthreads();
        sp[threadIdx.x] += ap;
        sf[threadIdx.x] += af;
        __syncthreads();
    }
    int64_t rp = sp[threadIdx.x] - tp, rf = sf[threadIdx.x] - tf;
    for (int64_t x = b; x < e; ++x) {
        const int64_t cp = poff[x], cf = foff[x];
        poff[x] = rp; foff[x] = rf;
        rp += cp; rf += cf;
    }
    if (threadIdx.x == 1023) { poff[nl] = sp[1023]; foff[nl] = sf[1023]; }
}

// largest l in [0, nl) with off[l] <= x
__device__ __forceinline__ int64_t plan_find(const int64_t* off, int64_t nl, int64_t x) {
    int64_t lo = 0, hi = nl - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (off[mid] <= x) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <int AGG, bool WAVE>
__global__ void __launch_bounds__(256) k_cnt_panes(TableView t, CountGeom G, const uint32_t* perm, const int64_t* val,
                                                   const int64_t* plan, const int64_t* poff, int64_t nl,
                                                   int64_t* tmp) {
    constexpr int W = (AGG == GW_AVG_I64 || AGG == GW_AVG_F64) ? 2 : 1;
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t gp = WAVE ? tid / 64 : tid;
    const int lane = WAVE ? (int)(threadIdx.x & 63) : 0;
    if (gp >= poff[nl]) return;  // the grid is an upper bound; WAVE: whole waves leave together
    const int64_t l = plan_find(poff, nl, gp);
    const int64_t* p = plan + l * kPlanWords;
    const int64_t i = p[kPlanI], L = p[kPlanL], c0 = p[kPlanC0];
    const int64_t g = G.g;
    const int64_t q = c0 / g + (gp - poff[l]);
    const int64_t o_lo = max(q * g, c0), o_hi = min((q + 1) * g, c0 + L);
    int64_t a0 = 0, a1 = 0;
    bool has = false;
    if (lane == 0 && o_lo > q * g) {  // the pane began before the batch: its ring cell
        const int64_t* e = slot_ptr(t, p[kPlanSlot]) + 2 + (q % t.ring) * W;
        a0 = e[0];
        a1 = W == 2 ? e[1] : 0;
        has = true;
    }
    for (int64_t o = o_lo + lane; o < o_hi; o += WAVE ? 64 : 1) {
        int64_t b0, b1;
        record_cell(AGG, val ? val[perm[i + (o - c0)]] : 0, b0, b1);
        if (has) fold_cell(AGG, a0, a1, b0, b1); else { a0 = b0; a1 = b1; has = true; }
    }
    if (WAVE) {
        for (int s = 1; s < 64; s <<= 1) {
            const int64_t b0 = __shfl_xor(a0, s), b1 = __shfl_xor(a1, s);
            const bool bh = __shfl_xor((int)has, s) != 0;
            if (bh) {
                if (has) fold_cell(AGG, a0, a1, b0, b1); else { a0 = b0; a1 = b1; has = true; }
            }
        }
    }
    if (lane == 0) {
        tmp[gp * W] = a0;
        if (W == 2) tmp[gp * W + 1] = a1;
    }
}

template <int AGG>
__global__ void __launch_bounds__(256) k_cnt_fires(TableView t, CountGeom G, const int64_t* plan, const int64_t* poff,
                                                   const int64_t* foff, int64_t nl, const int64_t* tmp,
                                                   int64_t* ok, int64_t* os, int64_t* oe, int64_t* orr, DevStatus* st) {
    constexpr int W = (AGG == GW_AVG_I64 || AGG == GW_AVG_F64) ? 2 : 1;
    const int64_t gf = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (gf >= foff[nl]) return;  // the grid is an upper bound
    const int64_t l = plan_find(foff, nl, gf);
    const int64_t* p = plan + l * kPlanWords;
    const int64_t c0 = p[kPlanC0], g = G.g;
    const int64_t pf = c0 / g;
    const int64_t* sp = slot_ptr(t, p[kPlanSlot]);
    const int64_t* cells = sp + 2;
    const int64_t* pv = tmp + poff[l] * W;
    const int64_t c = (c0 / G.slide + 1 + (gf - foff[l])) * G.slide;
    const int64_t len = c < G.size ? c : G.size;
    const int64_t p0 = (c - len) / g, p1 = c / g;
    auto pane = [&](int64_t q, int64_t& a, int64_t& b) {
        const int64_t* e = q >= pf ? pv + (q - pf) * W : cells + (q % t.ring) * W;
        a = e[0];
        b = W == 2 ? e[1] : 0;
    };
    int64_t r0, r1;
    pane(p0, r0, r1);
    for (int64_t q = p0 + 1; q < p1; ++q) {
        int64_t b0, b1;
        pane(q, b0, b1);
        fold_cell(AGG, r0, r1, b0, b1);
    }
    cnt_emit<AGG>(st, ok, os, oe, orr, sp[0], c, len, r0, r1);
}

__global__ void __launch_bounds__(256) k_cnt_ring(TableView t, CountGeom G, const int64_t* plan, const int64_t* poff,
                                                  int64_t nl, const int64_t* tmp) {
    const int R = t.ring, W = t.words;
    const int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (x >= nl * R) return;
    const int64_t l = x / R;
    const int q = (int)(x % R);
    const int64_t* p = plan + l * kPlanWords;
    const int64_t c0 = p[kPlanC0], L = p[kPlanL];
    const int64_t pf = c0 / G.g, pe = (c0 + L - 1) / G.g;
    int64_t* sp = slot_ptr(t, p[kPlanSlot]);
    const int64_t P = pe - q;
    if (P >= pf) {
        const int64_t* v = tmp + (poff[l] + (P - pf)) * W;
        int64_t* e = sp + 2 + (P % R) * W;
        for (int w = 0; w < W; ++w) e[w] = v[w];
    }
    if (q == 0) sp[1] = c0 + L;
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
    TableView tv{};          // main table (sessions: K1 inline; count windows: the pane ring)
    TableView wv{};          // wide table (sessions of keys with more than K1 in flight)
    DevStatus* d_st = nullptr;
    DevStatus* h_st = nullptr;
    uint32_t* slot[2] = {nullptr, nullptr};  // per record: slot (sort keys, double buffer)
    uint32_t* perm[2] = {nullptr, nullptr};  // per record: arrival index (sort values)
    uint32_t* r0 = nullptr;  // punted / retried run heads
    uint32_t* r1 = nullptr;
    int64_t* mig = nullptr;  // migration lists (main pass -> wide table)
    int64_t* rec = nullptr;  // sessions: (ts, value) per record
    // region-partitioned ingest (k_sp_*): pass-1 records (SoA), descriptor rows / columns,
    // punted records
    int64_t* sp_col3 = nullptr;  // key | ts | value, sp_cap each
    uint32_t* sp_row = nullptr;  // sp_desc_cap each: rows, then columns
    int64_t* pu_col3 = nullptr;  // punted key | ts | value, sp_cap each
    uint32_t* sp_grp = nullptr;  // grouping: offsets by position | offsets in order | heads, counts
    int64_t sp_cap = 0, sp_desc_cap = 0, sp_grp_cap = 0;
    int sp_key_grid = 0;
    bool fresh = false;      // h_st matches the device (nothing launched since the last refresh)
    int gshift = 0;          // sessions: the last sort grouped records by slot >> gshift
    uint32_t* due_list = nullptr;  // fire sweep: main-table slots with something due
    int64_t due_list_cap = 0;
    int64_t* cnt_plan = nullptr;  // count windows: long-run plan rows + pane / firing offsets
    int64_t cnt_plan_cap = 0;
    int64_t* cnt_tmp = nullptr;   // count windows: pane values of the long runs
    int64_t cnt_tmp_cap = 0;
    void* sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    int64_t buf_cap = 0;
    int64_t* o_key = nullptr;
    int64_t* o_start = nullptr;
    int64_t* o_end = nullptr;
    int64_t* o_res = nullptr;
    int64_t o_cap = 0;
    int64_t* lo_buf[3] = {nullptr, nullptr, nullptr};  // late side output: key | ts | value
    int64_t lo_cap = 0, lo_head = 0;
    int64_t wm = INT64_MIN;
    gw_stats stats{};
    bool timing = false;
    bool count_mode = false;  // GW_COUNT_TUMBLING / GW_COUNT_SLIDING (same slot table and row plumbing)
    CountGeom cg{};
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
    s->fresh = false;
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
    s->fresh = true;
    return GW_OK;
}

// Entry of a call that launches work: the host view is refreshed unless nothing ran on the
// device since the last refresh (the ingest and fire calls end with one).
static int begin_launch(SessionState* s, std::string& err) {
    int rc = s->fresh ? GW_OK : session_refresh(s, err);
    s->fresh = false;
    return rc;
}

// Zero a device status word without a host round trip (host view updated alike).
static int zero_word_async(SessionState* s, size_t off, std::string& err) {
    *reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(s->h_st) + off) = 0;
    SCHECK(hipMemsetAsync(reinterpret_cast<char*>(s->d_st) + off, 0, 8, s->stream));
    return GW_OK;
}

static int set_word(SessionState* s, size_t off, unsigned long long v, std::string& err) {
    unsigned long long* hv = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(s->h_st) + off);
    *hv = v;
    SCHECK(hipMemcpyAsync(reinterpret_cast<char*>(s->d_st) + off, hv, 8, hipMemcpyHostToDevice, s->stream));
    SCHECK(hipStreamSynchronize(s->stream));
    return GW_OK;
}

// ring = sessions (or count panes) per slot, words = int64 words each
static int alloc_table(SessionState* s, TableView& t, int64_t cap, int ring, int words, std::string& err) {
    t = s->tv;
    t.cap = cap;
    t.ring = ring;
    t.words = words;
    t.stride_w = (int)(((2 + ring * words) + 7) / 8 * 8);
    SCHECK(hipMalloc((void**)&t.base, (size_t)(cap + 1) * (t.stride_w + 1) * 8));  // slots + due times
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
    s->wv.agg = cfg.agg;
    std::string& err = why;
    SCHECK(hipMalloc((void**)&s->d_st, sizeof(DevStatus)));
    SCHECK(hipHostMalloc((void**)&s->h_st, sizeof(DevStatus), hipHostMallocDefault));
    SCHECK(hipMemset(s->d_st, 0, sizeof(DevStatus)));
    memset(s->h_st, 0, sizeof(DevStatus));
    int rc;
    if (cfg.assigner == GW_COUNT_TUMBLING || cfg.assigner == GW_COUNT_SLIDING) {
        s->count_mode = true;
        const int64_t size = cfg.size, slide = cfg.assigner == GW_COUNT_SLIDING ? cfg.slide : cfg.size;
        int64_t a = size, b = slide;
        while (b) { const int64_t t = a % b; a = b; b = t; }
        s->cg = CountGeom{size, slide, a};
        rc = alloc_table(s, s->tv, cap, (int)(size / a), cell_words(cfg.agg), why);  // ring of size/g panes
        if (rc) { session_destroy(s); return rc; }
        out = s;
        return GW_OK;
    }
    // K1 so that the slot is one 64-byte line: 2 sessions (sum/count/min/max), 1 (avg)
    const int words = cell_words(cfg.agg) == 2 ? 4 : 3;
    rc = alloc_table(s, s->tv, cap, words == 3 ? 2 : 1, words, why);
    if (rc == GW_OK) rc = alloc_table(s, s->wv, 1024, 4, kWideWords, why);
    if (rc) { session_destroy(s); return rc; }
    out = s;
    return GW_OK;
}

void session_destroy(SessionState* s) {
    if (!s) return;
    hipStreamSynchronize(s->stream);
    hipFree(s->tv.base);
    hipFree(s->wv.base);
    hipFree(s->d_st);
    hipHostFree(s->h_st);
    for (int q = 0; q < 2; ++q) { hipFree(s->slot[q]); hipFree(s->perm[q]); }
    hipFree(s->r0); hipFree(s->r1); hipFree(s->mig); hipFree(s->rec);
    hipFree(s->cnt_plan); hipFree(s->cnt_tmp); hipFree(s->due_list);
    hipFree(s->sort_tmp);
    hipFree(s->sp_col3); hipFree(s->sp_row); hipFree(s->pu_col3); hipFree(s->sp_grp);
    hipFree(s->o_key); hipFree(s->o_start); hipFree(s->o_end); hipFree(s->o_res);
    for (auto* p : s->lo_buf) hipFree(p);
    for (int w = 0; w < 2; ++w) for (auto& p : s->ev_pending[w]) s->ev_pool.push_back(p);
    for (auto& p : s->ev_pool) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
    delete s;
}

static int ensure_bufs(SessionState* s, int64_t n, std::string& err) {
    if (n <= s->buf_cap) return GW_OK;
    const int64_t c = std::max<int64_t>(n + n / 4, 1 << 16);
    SCHECK(hipStreamSynchronize(s->stream));
    for (int q = 0; q < 2; ++q) { hipFree(s->slot[q]); hipFree(s->perm[q]); }
    hipFree(s->r0); hipFree(s->r1); hipFree(s->mig); hipFree(s->sort_tmp); hipFree(s->rec);
    s->mig = nullptr;
    s->rec = nullptr;
    for (int q = 0; q < 2; ++q) {
        SCHECK(hipMalloc((void**)&s->slot[q], c * 4));
        SCHECK(hipMalloc((void**)&s->perm[q], c * 4));
    }
    SCHECK(hipMalloc((void**)&s->r0, c * 4));
    SCHECK(hipMalloc((void**)&s->r1, c * 4));
    if (!s->count_mode) SCHECK(hipMalloc((void**)&s->mig, (size_t)c * (2 + kWideWords * kLaneSess) * 8));
    if (!s->count_mode) SCHECK(hipMalloc((void**)&s->rec, (size_t)c * 16));
    rocprim::double_buffer<uint32_t> kb(s->slot[0], s->slot[1]), vb(s->perm[0], s->perm[1]);
    size_t bytes = 0;
    SCHECK(rocprim::radix_sort_pairs<SlotSortConfig>(nullptr, bytes, kb, vb, (size_t)c, 0, 32, s->stream));
    SCHECK(hipMalloc(&s->sort_tmp, bytes));
    s->sort_tmp_bytes = bytes;
    s->buf_cap = c;
    return GW_OK;
}

// Records of the batch, grouped by slot in arrival order: stable LSD radix sort of (slot,
// arrival index) over the slot bits.  Returns the sorted buffers.
static int sort_by_slot(SessionState* s, int64_t n, int64_t cap, const uint32_t** sk, const uint32_t** sp,
                        std::string& err) {
    int bits = 1;
    while (bits < 32 && ((uint64_t)(cap + 1) >> bits)) ++bits;
    // sessions may group by slot >> gshift so that the sort covers fewer bits (passes of 8);
    // the replay then separates the <= 2^gshift slots of a group (count windows need whole
    // slots).  Measured on 12.5M keys (26 slot bits): 24-bit groups save 80 us of sort but
    // cost 180 us of replay, so the default sorts whole slots; GW_SESSION_SORT_BITS sets
    // the cap (the tests force 4-bit groups)
    int sort_bits = 32;
    if (const char* e = getenv("GW_SESSION_SORT_BITS")) sort_bits = std::max(1, atoi(e));
    s->gshift = s->count_mode ? 0 : std::min(4, std::max(0, bits - sort_bits));
    rocprim::double_buffer<uint32_t> kb(s->slot[0], s->slot[1]), vb(s->perm[0], s->perm[1]);
    size_t bytes = s->sort_tmp_bytes;
    SCHECK(rocprim::radix_sort_pairs<SlotSortConfig>(s->sort_tmp, bytes, kb, vb, (size_t)n, s->gshift, bits, s->stream));
    *sk = kb.current();
    *sp = vb.current();
    return GW_OK;
}

// Grow a table to new_cap slots (and/or new ring): rehash its state into a fresh table.
static int regrow(SessionState* s, TableView& t, int64_t new_cap, int new_ring, bool wide, std::string& err) {
    TableView nt;
    int rc = alloc_table(s, nt, new_cap, new_ring, t.words, err);
    if (rc) return rc;
    if (wide) {
        SCHECK(launch_status_set(s->d_st, offsetof(DevStatus, pad[2]) / 8, 0, -1, s->stream));
    } else {
        SCHECK(launch_status_set(s->d_st, 0, 0, 1, s->stream));  // zero sh[].ins (used slots)
    }
    const int wps = s->count_mode ? t.ring * t.words : (wide ? -1 : t.ring * t.words);
    hipLaunchKernelGGL(k_sess_rehash, dim3(grid_of(t.cap + 1)), dim3(256), 0, s->stream, t, nt, wps, s->d_st,
                       wide ? -1 : 1);
    SCHECK(hipGetLastError());
    SCHECK(hipStreamSynchronize(s->stream));
    hipFree(t.base);
    t = nt;
    s->stats.rehashes++;
    rc = session_refresh(s, err);
    if (rc) return rc;
    if (s->h_st->flags & GW_DF_TABLE_FULL) { err = "session state table rehash overflow"; return GW_E_OOM; }
    return GW_OK;
}

// Room for `add` more wide keys (load <= 0.7) and lists of `need` sessions.
static int ensure_wide(SessionState* s, int64_t add, int64_t need, std::string& err) {
    const int64_t used = (int64_t)s->h_st->pad[2];
    int64_t cap = s->wv.cap;
    while ((double)(used + add) > 0.7 * (double)cap) cap *= 2;
    int ring = s->wv.ring;
    while (ring < need) ring *= 2;
    if (cap == s->wv.cap && ring == s->wv.ring) return GW_OK;
    return regrow(s, s->wv, cap, ring, true, err);
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

// Slot per record and the stable grouping by slot (both modes).  Grows the main table to
// keep its load below 0.7 for `n` possible new keys.
static int group_records(SessionState* s, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val,
                         const uint32_t** sk, const uint32_t** sp, std::string& err) {
    int rc;
    if ((double)(s->h_st->used_slots + n) > 0.7 * (double)s->tv.cap &&
        ((double)s->h_st->used_slots > 0.7 * (double)s->tv.cap ||
         (double)(s->h_st->used_slots + n) > 0.95 * (double)s->tv.cap)) {
        int64_t want = s->tv.cap;
        while ((double)(s->h_st->used_slots + n) > 0.7 * (double)want) want *= 2;
        if ((rc = regrow(s, s->tv, want, s->tv.ring, false, err))) return rc;
    }
    if ((rc = ensure_bufs(s, n, err))) return rc;
    for (int attempt = 0;; ++attempt) {
        hipLaunchKernelGGL(k_sess_prep, dim3(grid_of(n)), dim3(256), 0, s->stream, key, ts, val, n, s->tv, s->slot[0],
                           s->perm[0], s->count_mode ? nullptr : s->rec, s->d_st);
        if ((rc = session_refresh(s, err))) return rc;
        if (!(s->h_st->flags & GW_DF_TABLE_FULL)) break;
        if (attempt > 4) { err = "session state table full"; return GW_E_OOM; }
        SCHECK(launch_status_set(s->d_st, 0, 0, 2, s->stream));  // zero sh[].flags
        if ((rc = regrow(s, s->tv, s->tv.cap * 2, s->tv.ring, false, err))) return rc;
    }
    return sort_by_slot(s, n, s->tv.cap, sk, sp, err);
}

// Count windows: short runs one thread each, hot keys' long runs one workgroup each.
static int launch_count_apply(SessionState* s, const uint32_t* ks, const uint32_t* perm, int64_t n, const int64_t* val,
                              std::string& err) {
    int rc;
    if ((rc = zero_word_async(s, offsetof(DevStatus, overflow), err))) return rc;
    const int64_t* v = s->cfg.agg == GW_COUNT ? nullptr : val;
#define L(A)                                                                                               \
    hipLaunchKernelGGL(k_cnt_apply<A>, dim3(grid_of(n)), dim3(256), 0, s->stream, s->tv, s->cg, ks, perm, n, v, \
                       s->o_key, s->o_start, s->o_end, s->o_res, s->r0, s->d_st)
    GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
    SCHECK(hipGetLastError());
    if ((rc = session_refresh(s, err))) return rc;
    const int64_t nl = (int64_t)s->h_st->overflow;
    if (!nl) return GW_OK;
    // plan rows of the long runs, their pane / firing offsets (device scan), then the three
    // launches over upper bounds of the pane and firing counts (no host round trip)
    const int64_t pw = nl * kPlanWords + 2 * (nl + 1);
    if (pw > s->cnt_plan_cap) {
        SCHECK(hipStreamSynchronize(s->stream));
        hipFree(s->cnt_plan);
        s->cnt_plan_cap = std::max<int64_t>(pw * 2, 4096);
        SCHECK(hipMalloc((void**)&s->cnt_plan, s->cnt_plan_cap * 8));
    }
    const CountGeom& G = s->cg;
    int64_t* dpo = s->cnt_plan + nl * kPlanWords;
    int64_t* dfo = dpo + nl + 1;
    hipLaunchKernelGGL(k_cnt_long_info, dim3(grid_of(nl)), dim3(256), 0, s->stream, s->tv, G, ks, n, s->r0, nl,
                       s->cnt_plan, dpo, dfo);
    hipLaunchKernelGGL(k_cnt_plan_scan, dim3(1), dim3(1024), 0, s->stream, dpo, dfo, nl);
    const int64_t np_max = n / G.g + 2 * nl, nf_max = n / G.slide + nl;
    const int W = s->tv.words;
    if (np_max * W > s->cnt_tmp_cap) {
        SCHECK(hipStreamSynchronize(s->stream));
        hipFree(s->cnt_tmp);
        s->cnt_tmp_cap = std::max<int64_t>(np_max * W + np_max * W / 2, 1 << 16);
        SCHECK(hipMalloc((void**)&s->cnt_tmp, s->cnt_tmp_cap * 8));
    }
    const bool wave = G.g >= 16;
    const unsigned pg = (unsigned)((np_max * (wave ? 64 : 1) + 255) / 256);
#define L(A)                                                                                                   \
    if (wave)                                                                                                  \
        hipLaunchKernelGGL((k_cnt_panes<A, true>), dim3(pg), dim3(256), 0, s->stream, s->tv, G, perm, v, s->cnt_plan, \
                           dpo, nl, s->cnt_tmp);                                                               \
    else                                                                                                       \
        hipLaunchKernelGGL((k_cnt_panes<A, false>), dim3(pg), dim3(256), 0, s->stream, s->tv, G, perm, v,      \
                           s->cnt_plan, dpo, nl, s->cnt_tmp);                                                  \
    if (nf_max > 0)                                                                                            \
        hipLaunchKernelGGL(k_cnt_fires<A>, dim3((unsigned)((nf_max + 255) / 256)), dim3(256), 0, s->stream, s->tv, G, \
                           s->cnt_plan, dpo, dfo, nl, s->cnt_tmp, s->o_key, s->o_start, s->o_end, s->o_res, s->d_st)
    GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
    hipLaunchKernelGGL(k_cnt_ring, dim3((unsigned)((nl * s->tv.ring + 255) / 256)), dim3(256), 0, s->stream, s->tv, G,
                       s->cnt_plan, dpo, nl, s->cnt_tmp);
    SCHECK(hipGetLastError());
    return GW_OK;
}

// Count windows: slot per record, stable grouping by slot, one in-order fold per key.
static int count_ingest(SessionState* s, int64_t n, const int64_t* key, const int64_t* val, std::string& err) {
    int rc;
    if ((rc = begin_launch(s, err))) return rc;
    if (n <= 0) return GW_OK;
    if ((int64_t)n > (int64_t)0x7fffffffLL) { err = "batch too large"; return GW_E_INVALID; }
    // every element fires at most one window
    if ((rc = ensure_rows(s, (int64_t)s->h_st->rows + n, err))) return rc;
    auto ev = s->timing ? get_ev(s) : std::pair<hipEvent_t, hipEvent_t>{};
    if (s->timing) SCHECK(hipEventRecord(ev.first, s->stream));
    const uint32_t* ks;
    const uint32_t* perm;
    if ((rc = group_records(s, n, key, nullptr, nullptr, &ks, &perm, err))) return rc;
    if ((rc = launch_count_apply(s, ks, perm, n, val, err))) return rc;
    if (s->timing) {
        SCHECK(hipEventRecord(ev.second, s->stream));
        s->ev_pending[0].push_back(ev);
    }
    if ((rc = session_refresh(s, err))) return rc;
    if (s->h_st->flags & GW_DF_TABLE_FULL) { err = "count-window state table overflow"; return GW_E_OOM; }
    return GW_OK;
}

// The fields of a main-pass launch that both ingest paths share; reserves output room
// (rows fired at once under allowed lateness, the late side output).
static int seg_common(SessionState* s, SegArgs& a, int64_t n, int64_t wm, std::string& err) {
    int rc;
    a.n = n;
    a.gap = s->cfg.gap;
    a.wm = wm;
    a.lateness = s->cfg.allowed_lateness;
    a.purge = a.lateness > 0 && s->cfg.trigger == GW_PURGING_EVENT_TIME_TRIGGER;
    a.st = s->d_st;
    if (a.lateness > 0) {  // an element fires at most one window at once
        if ((rc = ensure_rows(s, (int64_t)s->h_st->rows + n, err))) return rc;
        a.o_key = s->o_key; a.o_start = s->o_start; a.o_end = s->o_end; a.o_res = s->o_res;
    }
    if (s->cfg.flags & GW_FLAG_LATE_SIDE_OUTPUT) {
        if ((rc = ensure_late(s, (int64_t)s->h_st->n_late_out + n, err))) return rc;
        a.lo_key = s->lo_buf[0]; a.lo_ts = s->lo_buf[1]; a.lo_val = s->lo_buf[2];
    }
    a.t = s->tv;
    a.w = s->wv;
    a.mig = s->mig;
    return GW_OK;
}

// Finished lists of more than K1 sessions (st->pad[0] of them) move to the wide table.
static int run_migrate(SessionState* s, std::string& err) {
    int rc;
    const int64_t n_mig = (int64_t)s->h_st->pad[0];
    if (!n_mig) return GW_OK;
    if ((rc = ensure_wide(s, n_mig, (int64_t)s->h_st->pad[1], err))) return rc;
    hipLaunchKernelGGL(k_sess_migrate, dim3(grid_of(n_mig)), dim3(256), 0, s->stream, s->tv, s->wv, s->mig, n_mig,
                       s->cfg.allowed_lateness, s->d_st);
    SCHECK(hipGetLastError());
    if ((rc = session_refresh(s, err))) return rc;
    if (s->h_st->flags & GW_DF_TABLE_FULL) { err = "session wide table full"; return GW_E_OOM; }
    return GW_OK;
}

// Sort path: slot per record (k_sess_prep), stable radix sort by slot, one thread per key run
// (k_sess_segment), migrations, then the wide pass over punted runs.  Replays the punt list
// of the region path, and is the whole ingest under GW_SESSION_PATH=sort.
static int ingest_sorted(SessionState* s, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val,
                         int64_t wm, std::string& err) {
    int rc;
    SegArgs a{};
    if ((rc = group_records(s, n, key, ts, val, &a.slot, &a.perm, err))) return rc;
    a.rec = s->rec;
    a.gshift = s->gshift;
    a.key = key;
    a.ts = ts;
    a.val = val;
    if ((rc = seg_common(s, a, n, wm, err))) return rc;
    // main pass (st->overflow, pad[0], pad[1] were zeroed by k_sess_prep)
    s->h_st->overflow = s->h_st->pad[0] = s->h_st->pad[1] = 0;
    a.punt = s->r0;
    const int64_t per_block = (int64_t)kSegChunk * (kSegThreads / 64);
    const unsigned gs = (unsigned)((n + per_block - 1) / per_block);
#define L(A) hipLaunchKernelGGL(k_sess_segment<A>, dim3(gs), dim3(kSegThreads), 0, s->stream, a)
    GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
    SCHECK(hipGetLastError());
    if ((rc = session_refresh(s, err))) return rc;
    int64_t n_punt = (int64_t)s->h_st->overflow;
    if ((rc = run_migrate(s, err))) return rc;
    // wide pass over the punted runs; runs that do not fit K2 retry after widening
    uint32_t* rin = s->r0;
    uint32_t* rout = s->r1;
    for (int pass = 0; n_punt > 0; ++pass) {
        if (pass > 40) { err = "session wide table did not converge"; return GW_E_DEVICE; }
        if ((rc = ensure_wide(s, n_punt, 0, err))) return rc;
        if ((rc = zero_word_async(s, offsetof(DevStatus, overflow), err))) return rc;
        if ((rc = zero_word_async(s, offsetof(DevStatus, pad[1]), err))) return rc;
        a.t = s->tv;
        a.w = s->wv;
        a.runs = rin;
        a.n_runs = n_punt;
        a.retry = rout;
#define L(A) hipLaunchKernelGGL(k_sess_wide<A>, dim3(grid_of(n_punt)), dim3(256), 0, s->stream, a)
        GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
        SCHECK(hipGetLastError());
        if ((rc = session_refresh(s, err))) return rc;
        n_punt = (int64_t)s->h_st->overflow;
        if (n_punt) {
            SCHECK(launch_status_set(s->d_st, 0, 0, 2, s->stream));  // zero sh[].flags (TABLE_FULL of the wide table)
            if ((rc = ensure_wide(s, n_punt, (int64_t)s->h_st->pad[1], err))) return rc;
        }
        std::swap(rin, rout);
    }
    return GW_OK;
}

static void sp_opt_in(SessionState* s) {
    if (!s->sp_key_grid) {  // persistent replay grid: the resident workgroups, a multiple of 8
        int dev = 0, cus = 0, per = 0;
        hipGetDevice(&dev);
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
#define L(A) hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k_sp_keys<A>, kSpKeyThreads, 0)
        GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
        s->sp_key_grid = std::max(8, (std::max(cus, 1) * std::max(per, 1)) / 8 * 8);
    }
    static bool done = false;
    if (!done) {
        hipFuncSetAttribute((const void*)k_sp_part, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSpPartLds);
        hipFuncSetAttribute((const void*)k_sp_group, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kGrpLds);
        done = true;
    }
}

// Region path (k_sp_part / k_sp_transpose / k_sp_group / k_sp_keys), then migrations, then the sort
// path over the punted records.
static int ingest_region(SessionState* s, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val,
                         int64_t wm, std::string& err) {
    int rc;
    // room for n new keys, as group_records keeps it: every key of the batch finds a slot
    // within the probe limit unless the table is nearly full (the punt list takes those)
    if ((double)(s->h_st->used_slots + n) > 0.7 * (double)s->tv.cap &&
        ((double)s->h_st->used_slots > 0.7 * (double)s->tv.cap ||
         (double)(s->h_st->used_slots + n) > 0.95 * (double)s->tv.cap)) {
        int64_t want = s->tv.cap;
        while ((double)(s->h_st->used_slots + n) > 0.7 * (double)want) want *= 2;
        if ((rc = regrow(s, s->tv, want, s->tv.ring, false, err))) return rc;
    }
    if ((rc = ensure_bufs(s, n, err))) return rc;  // the migration list
    int lcap = 0;
    while (((int64_t)1 << lcap) < s->tv.cap) ++lcap;
    int bb = std::min(lcap, 10);
    if (lcap - bb > kGrpMaxHomeBits) bb = lcap - kGrpMaxHomeBits;  // the sort key's home bits
    if (bb > 10) return ingest_sorted(s, n, key, ts, val, wm, err);  // beyond 2^26 slots
    const int nb = 1 << bb;
    const int64_t ntiles = (n + kSpTile - 1) / kSpTile;
    const int64_t recs = ntiles * kSpTile;
    if (recs > s->sp_cap || (int64_t)nb * kGrpCap > s->sp_grp_cap || ntiles * nb > s->sp_desc_cap) {
        SCHECK(hipStreamSynchronize(s->stream));
        if (recs > s->sp_cap) {
            hipFree(s->sp_col3); hipFree(s->pu_col3);
            s->sp_col3 = nullptr; s->pu_col3 = nullptr;
            const int64_t c = std::max<int64_t>(recs + recs / 4, kSpTile * 16);
            SCHECK(hipMalloc((void**)&s->sp_col3, (size_t)c * 24));
            SCHECK(hipMalloc((void**)&s->pu_col3, (size_t)c * 28));  // + the slow-slot list (u32)
            s->sp_cap = c;
        }
        if ((int64_t)nb * kGrpCap > s->sp_grp_cap) {
            hipFree(s->sp_grp);
            s->sp_grp = nullptr;
            const int64_t c = (int64_t)nb * kGrpCap;
            SCHECK(hipMalloc((void**)&s->sp_grp, (size_t)(3 * c + 2 * nb) * 4));  // offsets by position, order, heads
            s->sp_grp_cap = c;
        }
        if (ntiles * nb > s->sp_desc_cap) {
            hipFree(s->sp_row);
            s->sp_row = nullptr;
            const int64_t c = std::max<int64_t>((ntiles + ntiles / 4 + 16) * nb, 1 << 16);
            SCHECK(hipMalloc((void**)&s->sp_row, (size_t)c * 2 * 4));
            s->sp_desc_cap = c;
        }
    }
    const int64_t C = s->sp_cap, G = s->sp_grp_cap;
    int64_t* pk = s->sp_col3;
    uint32_t* row = s->sp_row;
    uint32_t* col = s->sp_row + s->sp_desc_cap;
    uint32_t* gsrc = s->sp_grp;
    uint32_t* perm = gsrc + G;
    uint32_t* shd = perm + G;
    uint32_t* grp_n = shd + G;
    sp_opt_in(s);
    if ((rc = zero_word_async(s, offsetof(DevStatus, overflow), err))) return rc;
    if ((rc = zero_word_async(s, offsetof(DevStatus, pad[0]), err))) return rc;
    if ((rc = zero_word_async(s, offsetof(DevStatus, pad[1]), err))) return rc;
    hipLaunchKernelGGL(k_sp_part, dim3((unsigned)ntiles), dim3(kSpThreads), kSpPartLds, s->stream, key, ts, val, n,
                       s->tv.cap, lcap, bb, pk, reinterpret_cast<longlong2*>(pk + C), row, s->d_st);
    hipLaunchKernelGGL(k_sp_transpose, dim3((unsigned)((ntiles + 63) / 64), (unsigned)((nb + 63) / 64)), dim3(256), 0,
                       s->stream, row, col, ntiles, nb);
    SCHECK(hipGetLastError());
    SegArgs a{};
    if ((rc = seg_common(s, a, n, wm, err))) return rc;
    a.p_key = pk;
    a.p_tv = reinterpret_cast<const longlong2*>(pk + C);
    a.col = col;
    a.ntiles = ntiles;
    a.lcap = lcap;
    a.bb = bb;
    a.pu_key = s->pu_col3;
    a.pu_ts = s->pu_col3 + C;
    a.pu_val = s->pu_col3 + 2 * C;
    static const int sp_exp = getenv("GW_SP_EXP") ? atoi(getenv("GW_SP_EXP")) : 0;
    a.exp = sp_exp;
    hipLaunchKernelGGL(k_sp_group, dim3((unsigned)nb), dim3(kGrpThreads), kGrpLds, s->stream, a, gsrc, perm, shd, grp_n);
    a.slow = reinterpret_cast<uint32_t*>(s->pu_col3 + 3 * C);
    if ((rc = zero_word_async(s, offsetof(DevStatus, spills), err))) return rc;
#define L(A)                                                                                                   \
    hipLaunchKernelGGL(k_sp_keys<A>, dim3((unsigned)s->sp_key_grid), dim3(kSpKeyThreads), 0, s->stream, a, perm, shd, \
                       grp_n, nb);                                                                              \
    hipLaunchKernelGGL(k_sp_slow<A>, dim3(1024), dim3(kSpKeyThreads), 0, s->stream, a, perm, shd, grp_n)
    GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
    SCHECK(hipGetLastError());
    if ((rc = session_refresh(s, err))) return rc;
    const int64_t n_punt = (int64_t)s->h_st->overflow;
    s->stats.session_punted += n_punt;
    if (sp_exp) {
        fprintf(stderr, "[sp_keys] slow home slots %llu of batch %lld (keys %llu, probe %llu, wide %llu, lane %llu), "
                        "punted %lld\n",
                (unsigned long long)s->h_st->spills, (long long)n, (unsigned long long)s->h_st->sh[0].pad0,
                (unsigned long long)s->h_st->sh[0].pad1, (unsigned long long)s->h_st->sh[1].pad0,
                (unsigned long long)s->h_st->sh[1].pad1, (long long)n_punt);
        SCHECK(launch_status_set(s->d_st, 0, 0, 6, s->stream));  // ShardCtr pad0
        SCHECK(launch_status_set(s->d_st, 0, 0, 7, s->stream));  // ShardCtr pad1
    }
    s->stats.session_slow += (int64_t)s->h_st->spills;
    if ((rc = run_migrate(s, err))) return rc;
    if (!n_punt) return GW_OK;
    hipLaunchKernelGGL(k_sp_unpunt, dim3(grid_of(n_punt)), dim3(256), 0, s->stream, s->tv, a.pu_key, n_punt);
    SCHECK(hipGetLastError());
    return ingest_sorted(s, n_punt, a.pu_key, a.pu_ts, a.pu_val, wm, err);
}

// GW_SESSION_PATH=region|sort picks the ingest path (GW_SESSION_SORT_BITS, the sort path's
// group tests, implies sort).
static bool region_ingest_enabled() {
    const char* p = getenv("GW_SESSION_PATH");
    if (p) return strcmp(p, "sort") != 0;
    return getenv("GW_SESSION_SORT_BITS") ? false : kSessionRegionDefault != 0;
}

int session_ingest(SessionState* s, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val, int64_t wm,
                   std::string& err) {
    if (s->count_mode) return count_ingest(s, n, key, val, err);
    int rc;
    if ((rc = begin_launch(s, err))) return rc;
    if (n <= 0) return GW_OK;
    if ((int64_t)n > (int64_t)0x7fffffffLL) { err = "batch too large"; return GW_E_INVALID; }
    auto ev = s->timing ? get_ev(s) : std::pair<hipEvent_t, hipEvent_t>{};
    if (s->timing) SCHECK(hipEventRecord(ev.first, s->stream));
    rc = region_ingest_enabled() ? ingest_region(s, n, key, ts, val, wm, err) : ingest_sorted(s, n, key, ts, val, wm, err);
    if (rc) return rc;
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
    if ((rc = begin_launch(s, err))) return rc;
    const int64_t before = (int64_t)s->h_st->rows;
    const int64_t need = before + (int64_t)(s->h_st->used_slots + 1) * s->tv.ring +
                         (int64_t)(s->h_st->pad[2] + 1) * s->wv.ring;
    if ((rc = ensure_rows(s, need, err))) return rc;
    auto ev = s->timing ? get_ev(s) : std::pair<hipEvent_t, hipEvent_t>{};
    if (s->timing) SCHECK(hipEventRecord(ev.first, s->stream));
    const unsigned fg = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(1, (s->tv.cap + 1 + 255) / 256));
    if (s->due_list_cap < s->tv.cap + 1) {
        hipFree(s->due_list);
        s->due_list = nullptr;
        SCHECK(hipMalloc((void**)&s->due_list, (size_t)(s->tv.cap + 1) * 4));
        s->due_list_cap = s->tv.cap + 1;
    }
    if ((rc = zero_word_async(s, offsetof(DevStatus, n_refire), err))) return rc;  // due-list cursor
    const unsigned sg = (unsigned)std::min<int64_t>(2048, std::max<int64_t>(1, (s->tv.cap + 1) / 2048));
    hipLaunchKernelGGL(k_sess_due_scan, dim3(sg), dim3(256), 0, s->stream, s->tv, wm, s->due_list, s->d_st);
    const int purge = (int)(s->cfg.allowed_lateness > 0 && s->cfg.trigger == GW_PURGING_EVENT_TIME_TRIGGER);
#define L(A)                                                                                               \
    hipLaunchKernelGGL(k_sess_fire<A>, dim3(fg), dim3(256), 0, s->stream, s->tv, s->due_list, wm,            \
                       s->cfg.allowed_lateness, purge, s->o_key, s->o_start, s->o_end, s->o_res, s->d_st); \
    if (s->h_st->pad[2])                                                                                    \
    hipLaunchKernelGGL(k_sess_fire_wide<A>, dim3(grid_of(s->wv.cap + 1)), dim3(256), 0, s->stream, s->wv, wm, \
                       s->cfg.allowed_lateness, purge, s->o_key, s->o_start, s->o_end, s->o_res, s->d_st)
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
// (key, start, end, a0, a1, fired) entry per session.
int session_collect(SessionState* s, int32_t kg_lo, int32_t kg_hi, std::vector<int64_t>& ent,
                    std::vector<int32_t>& kgs, std::string& err, const std::function<int32_t(int64_t)>& hash_of) {
    SCHECK(hipStreamSynchronize(s->stream));
    for (int tab = 0; tab < (s->count_mode ? 1 : 2); ++tab) {
        const TableView& t = tab ? s->wv : s->tv;
        const size_t words = (size_t)(t.cap + 1) * t.stride_w;
        std::vector<int64_t> h(words);
        SCHECK(hipMemcpy(h.data(), t.base, words * 8, hipMemcpyDeviceToHost));
        const int SW = t.words;
        for (int64_t i = 0; i <= t.cap; ++i) {
            const int64_t* sp = h.data() + (size_t)i * t.stride_w;
            if (sp[1] == 0) continue;
            if (tab == 0 && !s->count_mode && ((uint64_t)sp[1] & kBigMeta)) continue;  // in the wide table
            const int64_t key = i == t.cap ? kEmptyKey : sp[0];
            const int32_t kg = key_group_for_hash(hash_of ? hash_of(key) : java_long_hash(key), s->cfg.max_parallelism);
            if (kg < kg_lo || kg > kg_hi) continue;
            if (s->count_mode) {  // (key, element count, ring of pane accumulators)
                ent.push_back(key);
                ent.insert(ent.end(), sp + 1, sp + 2 + t.ring * SW);
                kgs.push_back(kg);
                continue;
            }
            const int cnt = tab ? (int)sp[1] : (int)((uint64_t)sp[1] & 0x7fffffffull);
            for (int q = 0; q < cnt; ++q) {
                const int64_t* x = sp + 2 + q * SW;
                int64_t e[6];
                if (tab) {
                    e[0] = key; e[1] = x[0]; e[2] = x[1]; e[3] = x[2]; e[4] = x[3]; e[5] = x[4] != 0;
                } else {
                    const int64_t fired = (int64_t)(((uint64_t)sp[1] >> (32 + q)) & 1ull);  // kept under lateness
                    e[0] = key; e[1] = x[0]; e[2] = x[1]; e[3] = x[2]; e[4] = SW == 4 ? x[3] : 0; e[5] = fired;
                }
                ent.insert(ent.end(), e, e + 6);
                kgs.push_back(kg);
            }
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
        if ((rc = regrow(s, s->tv, want, s->tv.ring, false, err))) return rc;
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
    int64_t maxk = 0, run = 0, wide = 0;
    for (int64_t j = 0; j < n; ++j) {
        const int64_t* x = ent + ord[j] * 6;
        if (j == 0 || x[0] != rk.back()) {
            if (j && run > s->tv.ring) wide++;
            rk.push_back(x[0]);
            roff.push_back(j);
            run = 0;
        }
        maxk = std::max(maxk, ++run);
        rs.insert(rs.end(), x + 1, x + 6);
    }
    if (run > s->tv.ring) wide++;
    roff.push_back(n);
    const int64_t nk = (int64_t)rk.size();
    if (wide && (rc = ensure_wide(s, wide, maxk, err))) return rc;
    if ((double)(s->h_st->used_slots + nk) > 0.7 * (double)s->tv.cap) {
        int64_t want = s->tv.cap;
        while ((double)(s->h_st->used_slots + nk) > 0.7 * (double)want) want *= 2;
        if ((rc = regrow(s, s->tv, want, s->tv.ring, false, err))) return rc;
    }
    int64_t *d_k = nullptr, *d_o = nullptr, *d_s = nullptr;
    SCHECK(hipMalloc((void**)&d_k, nk * 8));
    SCHECK(hipMalloc((void**)&d_o, (nk + 1) * 8));
    SCHECK(hipMalloc((void**)&d_s, n * 40));
    SCHECK(hipMemcpy(d_k, rk.data(), nk * 8, hipMemcpyHostToDevice));
    SCHECK(hipMemcpy(d_o, roff.data(), (nk + 1) * 8, hipMemcpyHostToDevice));
    SCHECK(hipMemcpy(d_s, rs.data(), n * 40, hipMemcpyHostToDevice));
    if ((rc = set_word(s, offsetof(DevStatus, overflow), 0, err))) return rc;
    hipLaunchKernelGGL(k_sess_restore, dim3(grid_of(nk)), dim3(256), 0, s->stream, s->tv, s->wv, d_k, d_o, d_s, nk,
                       s->cfg.allowed_lateness, s->d_st);
    SCHECK(hipGetLastError());
    rc = session_refresh(s, err);
    hipFree(d_k);
    hipFree(d_o);
    hipFree(d_s);
    if (rc) return rc;
    if (s->h_st->flags & GW_DF_TABLE_FULL) { err = "session state table full"; return GW_E_OOM; }
    if (s->h_st->overflow) {
        err = "a restored key already holds sessions in this operator (key group restored twice)";
        return GW_E_UNSUPPORTED;
    }
    return GW_OK;
}

int64_t session_late(SessionState* s) { return (int64_t)s->h_st->late; }

void session_stats(SessionState* s, gw_stats* out) {
    out->late_dropped = (int64_t)s->h_st->late;
    out->live_keys = (int64_t)s->h_st->used_slots;
    out->table_capacity = s->tv.cap;
    out->table_bytes = (int64_t)(s->tv.cap + 1) * s->tv.stride_w * 8 + (int64_t)(s->wv.cap + 1) * s->wv.stride_w * 8;
    out->session_merges = (int64_t)s->h_st->merges;
    out->fires = s->stats.fires;
    out->rehashes = s->stats.rehashes;
    out->session_punted = s->stats.session_punted;
    out->session_slow = s->stats.session_slow;
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
