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
// a stable radix sort by slot (gw_sort.hip) groups each key's records in ARRIVAL order, and one
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

namespace gw {

// Experiment builds only (flink_amd.build --define GW_SEG_EXP=n --out ...), results discarded:
// 1 no record gathers, 2 no slot write-back.  The product library is built with 0.
#ifndef GW_SEG_EXP
#define GW_SEG_EXP 0
#endif

constexpr int kLaneSess = 3;        // sessions a thread replays in LDS
constexpr int kSegThreads = 128;
constexpr int kWideWords = 5;       // wide-table session: start, end, a0, a1, fired
constexpr uint64_t kBigMeta = 1ull << 31;  // main-table slot word 1: the key lives in the wide table

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
    int64_t* pu_key;        // records of keys the prep found no slot for (arrival order), append at
                            // st->spills: replayed after a regrow
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

// Due summary: per block of kDueBlk slots a lower bound of their due times (after the due
// array), so the fire sweep reads 8 B per 64 slots and only the blocks that can hold
// something due.  Writers keep it a lower bound (atomicMin of a new due time); the sweep
// makes a block's entry exact again after scanning it.  INT64_MIN: scan the block.
constexpr int kDueBlkBits = 6;
constexpr int kDueBlk = 1 << kDueBlkBits;
__host__ __device__ __forceinline__ int64_t due_blocks(int64_t cap) { return (cap + 1 + kDueBlk - 1) >> kDueBlkBits; }
__device__ __forceinline__ int64_t* dsum_of(const TableView& t) { return due_of(t) + (t.cap + 1); }

// Dense key array beside the slot lines (after the due summary): a probe reads 8 B per slot
// instead of a 64-B slot line, so the probes of a batch touch cap x 8 B (268 MB at 2^25
// slots, mostly resident in the memory-side cache) rather than the whole table.  The slot
// line keeps its key word too (every reader of a slot's key uses it): a claimed slot gets
// its key in both places, the dense word first (the CAS), then the line.  Within the kernel
// that claims a slot another thread may find the key in the dense array before the line
// holds it; no kernel reads a line's key word in the launch that claims it.
__host__ __device__ __forceinline__ size_t table_words(int64_t cap, int stride_w) {
    return (size_t)(cap + 1) * (stride_w + 1) + (size_t)due_blocks(cap) + (size_t)(cap + 1);
}
__device__ __forceinline__ int64_t* keys_of(const TableView& t) { return dsum_of(t) + due_blocks(t.cap); }

__device__ __forceinline__ int64_t sess_find_or_insert(const TableView& t, int64_t key, bool& inserted) {
    inserted = false;
    if (key == kEmptyKey) return t.cap;  // sentinel slot
    int64_t* keys = keys_of(t);
    const uint64_t mask = (uint64_t)t.cap - 1;
    uint64_t idx = slot_hash(key) & mask;
    for (int p = 0; p < kMaxProbe; ++p) {
        const int64_t k = keys[idx];  // plain load: a stale read can only be kEmptyKey (the CAS resolves it)
        if (k == key) return (int64_t)idx;
        if (k == kEmptyKey) {
            const unsigned long long prev = atomicCAS((unsigned long long*)(keys + idx), (unsigned long long)kEmptyKey,
                                                      (unsigned long long)key);
            if (prev == (unsigned long long)kEmptyKey) {
                inserted = true;
                slot_ptr(t, (int64_t)idx)[0] = key;
                return (int64_t)idx;
            }
            if ((int64_t)prev == key) return (int64_t)idx;
        }
        idx = (idx + 1) & mask;
    }
    return -1;
}
__device__ __forceinline__ int64_t sess_find_slot(const TableView& t, int64_t key) {
    if (key == kEmptyKey) return t.cap;
    const int64_t* keys = keys_of(t);
    const uint64_t mask = (uint64_t)t.cap - 1;
    uint64_t idx = slot_hash(key) & mask;
    for (int p = 0; p < kMaxProbe; ++p) {
        const int64_t k = keys[idx];
        if (k == key) return (int64_t)idx;
        if (k == kEmptyKey) return -1;
        idx = (idx + 1) & mask;
    }
    return -1;
}
__device__ __forceinline__ void due_set(const TableView& t, int64_t slot, int64_t due) {
    due_of(t)[slot] = due;
    if (due == INT64_MAX) return;
    // only a lower due time changes the bound; within a kernel the bound only falls, so a
    // plain read that is stale is high, and costs no more than the atomic it then does
    long long* d = (long long*)dsum_of(t) + (slot >> kDueBlkBits);
    if ((long long)due < *d) atomicMin(d, (long long)due);
}

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
    const TsVal tv = (GW_SEG_EXP & 1) ? TsVal{a.wm + 1 + (int64_t)(idx & 7), 1} : reinterpret_cast<const TsVal*>(a.rec)[idx];
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
    if (GW_SEG_EXP & 2) return;
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
        due_set(a.t, slot, due);
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
    if ((int64_t)slot == a.t.cap + 1) {  // keys k_sess_prep found no slot for: replayed after a regrow
        unsigned long long at = atomicAdd(&a.st->spills, (unsigned long long)L);
        struct alignas(16) TsVal { int64_t ts, v; };
        for (int64_t r = i; r < j; ++r) {
            if (a.slot[r] != slot) continue;
            const uint32_t idx = a.perm[r];
            const TsVal tv = reinterpret_cast<const TsVal*>(a.rec)[idx];
            a.pu_key[at] = a.key[idx];
            a.pu_ts[at] = tv.ts;
            a.pu_val[at] = tv.v;
            ++at;
        }
        return;
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
    const int64_t g2 = sess_find_or_insert(w, key, inserted);
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
        const int64_t g2 = sess_find_or_insert(w, key, inserted);
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
        const int64_t g2 = sess_find_or_insert(a.w, key, inserted);
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
                                                   TableView t, uint32_t* slot, int64_t* rec,
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
        int64_t s = sess_find_or_insert(t, key[i], inserted);
        ins += inserted;
        if (s < 0) { flags |= GW_DF_TABLE_FULL; s = t.cap + 1; }  // no slot: sorts last, the segment punts it
        slot[i] = (uint32_t)s;  // (the arrival index, perm, is made by the sort's first pass)
        if (rec) {
            rec[2 * i] = ts[i];
            rec[2 * i + 1] = val ? val[i] : 0;
        }
    }
    block_commit(st, 0, ins, flags, 0);
}

// Fire sweep, part 1: list the slots with something due at `wm` -- a small fraction: the
// sessions that close at this watermark.  A wave reads the due summary of 64 blocks (one per
// lane), then scans each block whose lower bound is <= wm (64 due times, one per lane),
// lists its due slots and stores the block's exact minimum over the slots it did not list
// (k_sess_fire lowers it again for the slots it re-arms).  Hits are collected in LDS and
// list space is reserved with one atomic per workgroup.
constexpr int kDueBuf = 4096;
__global__ void __launch_bounds__(256) k_sess_due_scan(TableView t, int64_t wm, uint32_t* list, DevStatus* st) {
    __shared__ uint32_t buf[kDueBuf];
    __shared__ unsigned cnt;
    __shared__ unsigned long long gbase;
    // an ingest's follow-up (punts or migrations) is pending: the host fires again after it
    if (st->overflow | st->pad[0] | st->spills) return;
    const int64_t nslots = t.cap + 1, nblk = due_blocks(t.cap);
    const int64_t* due = due_of(t);
    int64_t* dsum = dsum_of(t);
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
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
    for (int64_t b0 = wave * 64; b0 < nblk; b0 += nwaves * 64) {
        const int64_t bl = b0 + lane;
        const bool hot = bl < nblk && dsum[bl] <= wm;
        for (uint64_t m = __ballot(hot); m; m &= m - 1) {  // wave-uniform
            const int64_t b = b0 + __ffsll((long long)m) - 1;
            const int64_t i = (b << kDueBlkBits) + lane;
            const int64_t d = i < nslots ? due[i] : INT64_MAX;
            const bool h = i < nslots && d <= wm;  // (wm may be Long.MAX_VALUE: the padding is never due)
            if (h) hit(i);
            int64_t mn = h ? INT64_MAX : d;
            for (int o = 32; o > 0; o >>= 1) mn = min(mn, (int64_t)__shfl_xor(mn, o));
            if (lane == 0) dsum[b] = mn;
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
            due_set(t, i, inline_due(s, SW, lateness));
        }
    }
    stage_flush(rs, &st->rows, o_key, o_start, o_end, o_res);
}

// The same for the wide table (one thread per wide slot; few keys).
template <int AGG>
__global__ void __launch_bounds__(256) k_sess_fire_wide(TableView w, int64_t wm, int64_t lateness, int purge,
                                                        int64_t* o_key, int64_t* o_start, int64_t* o_end,
                                                        int64_t* o_res, DevStatus* st) {
    if (st->overflow | st->pad[0] | st->spills) return;  // as k_sess_due_scan
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
        const int64_t j = sess_find_or_insert(n, key, inserted);
        if (j < 0) { flags |= GW_DF_TABLE_FULL; continue; }
        ins += inserted;
        int64_t* d = slot_ptr(n, j);
        d[1] = s[1];
        const int nw = words_per_slot < 0 ? (int)s[1] * o.words : words_per_slot;
        for (int w = 0; w < nw; ++w) d[2 + w] = s[2 + w];
        if (ins_field < 0) due_of(n)[j] = due_of(o)[i];
        else due_set(n, j, due_of(o)[i]);
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
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < due_blocks(t.cap);
         b += (int64_t)gridDim.x * blockDim.x)
        dsum_of(t)[b] = INT64_MAX;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= t.cap; i += (int64_t)gridDim.x * blockDim.x)
        keys_of(t)[i] = kEmptyKey;
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
        const int64_t slot = sess_find_or_insert(t, rk[i], inserted);
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
            due_set(t, slot, inline_due(sp, SW, lateness));
        } else {
            const int64_t g2 = sess_find_or_insert(w, rk[i], inserted);
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
        const int64_t j = sess_find_or_insert(t, e[0], inserted);
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
    int64_t* rec = nullptr;  // sessions: (ts, value) per record in arrival order
    int64_t* pu_rec = nullptr;  // sessions: records of keys the prep found no slot for, key | ts | value
    bool fresh = false;      // h_st matches the device (nothing launched since the last refresh)
    // An ingest whose host follow-up (sort_tail: migrations, the wide pass, records without a
    // slot) waits for the next sync: the fire launched right after it checks the device
    // counters and skips itself if the follow-up has work (k_sess_due_scan), so the common
    // batch costs one host sync, not two.
    bool sb_pend = false;
    SegArgs sort_a{};
    int64_t sb_wm = 0, sb_new = 0;
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

static int sb_finish(SessionState* s, std::string& err);

// Device counters -> host view (one host sync), then a pending ingest's follow-up.
static int sess_sync(SessionState* s, std::string& err) {
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

int session_refresh(SessionState* s, std::string& err) {
    int rc = sess_sync(s, err);
    if (rc == GW_OK && s->sb_pend) rc = sb_finish(s, err);
    return rc;
}

// Entry of a call that launches work: the host view is refreshed unless nothing ran on the
// device since the last refresh (the ingest and fire calls end with one).
static int begin_launch(SessionState* s, std::string& err) {
    int rc = s->fresh ? GW_OK : session_refresh(s, err);
    s->fresh = false;
    return rc;
}

// Zero a device status word without a host round trip (host view updated alike): one
// one-wave kernel (k_status_set, ~1 us) rather than a runtime fill (~5 us and more host time:
// ~14 per 10M-record sessions step, profiles/r6/configs/kernel_stats_sessions.csv).
static int zero_word_async(SessionState* s, size_t off, std::string& err) {
    *reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(s->h_st) + off) = 0;
    SCHECK(launch_status_set(s->d_st, (int)(off / 8), 0ull, -1, s->stream));
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
    SCHECK(hipMalloc((void**)&t.base, table_words(cap, t.stride_w) * 8));  // slots + due times + due summary + keys
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
    hipFree(s->r0); hipFree(s->r1); hipFree(s->mig); hipFree(s->rec); hipFree(s->pu_rec);
    hipFree(s->cnt_plan); hipFree(s->cnt_tmp); hipFree(s->due_list);
    hipFree(s->sort_tmp);
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
    hipFree(s->r0); hipFree(s->r1); hipFree(s->mig); hipFree(s->sort_tmp); hipFree(s->rec); hipFree(s->pu_rec);
    s->mig = nullptr;
    s->rec = nullptr;
    s->pu_rec = nullptr;
    for (int q = 0; q < 2; ++q) {
        SCHECK(hipMalloc((void**)&s->slot[q], c * 4));
        SCHECK(hipMalloc((void**)&s->perm[q], c * 4));
    }
    SCHECK(hipMalloc((void**)&s->r0, c * 4));
    SCHECK(hipMalloc((void**)&s->r1, c * 4));
    if (!s->count_mode) SCHECK(hipMalloc((void**)&s->mig, (size_t)c * (2 + kWideWords * kLaneSess) * 8));
    if (!s->count_mode) SCHECK(hipMalloc((void**)&s->rec, (size_t)c * 16));
    if (!s->count_mode) SCHECK(hipMalloc((void**)&s->pu_rec, (size_t)c * 24));
    const size_t bytes = (size_t)sort_scratch_bytes(c);
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
    int alt = 0;
    SCHECK(sort_pairs_u32(s->slot[0], s->perm[0], s->slot[1], s->perm[1], n, s->gshift, bits, s->sort_tmp, s->stream,
                          &alt, /*iota=*/true));
    *sk = s->slot[alt];
    *sp = s->perm[alt];
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
                         const uint32_t** sk, const uint32_t** sp, std::string& err, bool defer = false) {
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
                           s->count_mode ? nullptr : s->rec, s->d_st);
        // deferred (sessions): no host wait here; records without a slot sort last and the
        // segment punts them for a replay after a regrow (sort_tail)
        if (defer && !s->count_mode) break;
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
    if (n > kSortMaxRecords) { err = "batch too large for the grouping sort (split by the caller)"; return GW_E_INVALID; }
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
    // A key that finds no wide slot within the probe limit (hash-colliding keys) leaves its
    // entry; the table doubles and the whole list runs again (an entry already moved finds its
    // wide slot and is written again with the same contents).
    for (int attempt = 0;; ++attempt) {
        hipLaunchKernelGGL(k_sess_migrate, dim3(grid_of(n_mig)), dim3(256), 0, s->stream, s->tv, s->wv, s->mig, n_mig,
                           s->cfg.allowed_lateness, s->d_st);
        SCHECK(hipGetLastError());
        if ((rc = session_refresh(s, err))) return rc;
        if (!(s->h_st->flags & GW_DF_TABLE_FULL)) break;
        if (attempt >= 8) { err = "session wide table full"; return GW_E_OOM; }
        SCHECK(launch_status_set(s->d_st, 0, 0, 2, s->stream));  // zero sh[].flags
        s->h_st->flags &= ~GW_DF_TABLE_FULL;
        if ((rc = regrow(s, s->wv, s->wv.cap * 2, s->wv.ring, true, err))) return rc;
    }
    if ((rc = zero_word_async(s, offsetof(DevStatus, pad[0]), err))) return rc;  // (the fire's guard)
    return GW_OK;
}

// Session ingest: slot per record (k_sess_prep), stable radix sort by slot (gw_sort.hip), one
// thread per key run (k_sess_segment), migrations, then the wide pass over punted runs.
static int sort_tail(SessionState* s, SegArgs a, int64_t wm, std::string& err);

// defer: return right after the segment launch (no host wait) when the replay emits nothing
// (no allowed lateness, no side output); the tail -- migrations, the wide pass over punted
// runs, records without a slot -- runs at the next sync (sb_finish), and the watermark's fire
// launched before it skips itself on the device while that work is pending.
static int ingest_sorted(SessionState* s, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val,
                         int64_t wm, std::string& err, bool defer = false) {
    int rc;
    SegArgs a{};
    static const bool always = getenv("GW_SESSION_SYNC") && atoi(getenv("GW_SESSION_SYNC")) != 0;
    defer = defer && !always && s->cfg.allowed_lateness == 0 && !(s->cfg.flags & GW_FLAG_LATE_SIDE_OUTPUT);
    if ((rc = group_records(s, n, key, ts, val, &a.slot, &a.perm, err, defer))) return rc;
    a.rec = s->rec;
    a.gshift = s->gshift;
    a.key = key;
    a.ts = ts;
    a.val = val;
    if ((rc = seg_common(s, a, n, wm, err))) return rc;
    // main pass (st->overflow, pad[0], pad[1] were zeroed by k_sess_prep)
    s->h_st->overflow = s->h_st->pad[0] = s->h_st->pad[1] = 0;
    a.punt = s->r0;
    const int64_t C = s->buf_cap;  // records without a slot (deferred prep): punt columns
    a.pu_key = s->pu_rec;
    a.pu_ts = s->pu_rec + C;
    a.pu_val = s->pu_rec + 2 * C;
    const int64_t per_block = (int64_t)kSegChunk * (kSegThreads / 64);
    const unsigned gs = (unsigned)((n + per_block - 1) / per_block);
#define L(A) hipLaunchKernelGGL(k_sess_segment<A>, dim3(gs), dim3(kSegThreads), 0, s->stream, a)
    GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
    SCHECK(hipGetLastError());
    if (defer) {
        s->sort_a = a;
        s->sb_pend = true;
        s->sb_wm = wm;
        s->sb_new = n;
        s->fresh = false;
        return GW_OK;
    }
    if ((rc = session_refresh(s, err))) return rc;
    return sort_tail(s, a, wm, err);
}

// The slot sort path after its segment (h_st fresh): migrations, the wide pass over the
// punted runs, then the records whose keys found no slot (a deferred prep) after a regrow.
static int sort_tail(SessionState* s, SegArgs a, int64_t wm, std::string& err) {
    int rc;
    const int64_t n_fail = (int64_t)s->h_st->spills;
    if (n_fail > 0) {  // the prep's TABLE_FULL is handled below, not an error of the passes before
        s->stats.session_punted += n_fail;
        if ((rc = zero_word_async(s, offsetof(DevStatus, spills), err))) return rc;
        SCHECK(launch_status_set(s->d_st, 0, 0, 2, s->stream));  // zero sh[].flags
        s->h_st->flags &= ~GW_DF_TABLE_FULL;
    }
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
            // keys that found no wide slot within the probe limit (hash-colliding keys): a
            // bigger table spreads them, which the load rule alone would not ask for
            const bool full = (s->h_st->flags & GW_DF_TABLE_FULL) != 0;
            SCHECK(launch_status_set(s->d_st, 0, 0, 2, s->stream));  // zero sh[].flags (TABLE_FULL of the wide table)
            s->h_st->flags &= ~GW_DF_TABLE_FULL;
            if (full && (rc = regrow(s, s->wv, s->wv.cap * 2, s->wv.ring, true, err))) return rc;
            if ((rc = ensure_wide(s, n_punt, (int64_t)s->h_st->pad[1], err))) return rc;
        }
        std::swap(rin, rout);
    }
    if (n_fail > 0) {
        if ((rc = regrow(s, s->tv, s->tv.cap * 2, s->tv.ring, false, err))) return rc;
        if ((rc = ingest_sorted(s, n_fail, a.pu_key, a.pu_ts, a.pu_val, wm, err, false))) return rc;
    }
    return GW_OK;
}

// The deferred tail of the last ingest (h_st fresh): migrations, the wide pass, records
// without a slot (sort_tail).
static int sb_finish(SessionState* s, std::string& err) {
    if (!s->sb_pend) return GW_OK;
    s->sb_pend = false;
    return sort_tail(s, s->sort_a, s->sb_wm, err);
}

int session_ingest(SessionState* s, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val, int64_t wm,
                   std::string& err) {
    if (s->count_mode) return count_ingest(s, n, key, val, err);
    int rc;
    if ((rc = begin_launch(s, err))) return rc;
    if (n <= 0) return GW_OK;
    if (n > kSortMaxRecords) { err = "batch too large for the grouping sort (split by the caller)"; return GW_E_INVALID; }
    auto ev = s->timing ? get_ev(s) : std::pair<hipEvent_t, hipEvent_t>{};
    if (s->timing) SCHECK(hipEventRecord(ev.first, s->stream));
    if ((rc = ingest_sorted(s, n, key, ts, val, wm, err, true))) return rc;
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
    for (;;) {
        // spec: an ingest's follow-up is pending (its replay emitted no rows); this fire runs
        // before the host has looked, and skips itself on the device if there is follow-up work
        const bool spec = s->sb_pend;
        if (spec) {
            s->fresh = false;
        } else if ((rc = begin_launch(s, err))) {
            return rc;
        }
        const int64_t before = (int64_t)s->h_st->rows;
        const int64_t keys = (int64_t)s->h_st->used_slots + (spec ? s->sb_new : 0);  // spec: an upper bound
        const int64_t need = before + (keys + 1) * s->tv.ring + (int64_t)(s->h_st->pad[2] + 1) * s->wv.ring;
        if ((rc = ensure_rows(s, need, err))) return rc;
        auto ev = s->timing ? get_ev(s) : std::pair<hipEvent_t, hipEvent_t>{};
        if (s->timing) SCHECK(hipEventRecord(ev.first, s->stream));
        const unsigned fg = (unsigned)std::min<int64_t>(1024, std::max<int64_t>(1, (s->tv.cap + 1 + 255) / 256));
        if (s->due_list_cap < s->tv.cap + 1) {
            SCHECK(hipStreamSynchronize(s->stream));
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
        hipLaunchKernelGGL(k_sess_fire<A>, dim3(fg), dim3(256), 0, s->stream, s->tv, s->due_list, wm,        \
                           s->cfg.allowed_lateness, purge, s->o_key, s->o_start, s->o_end, s->o_res, s->d_st); \
        if (s->h_st->pad[2])                                                                                \
        hipLaunchKernelGGL(k_sess_fire_wide<A>, dim3(grid_of(s->wv.cap + 1)), dim3(256), 0, s->stream, s->wv, wm, \
                           s->cfg.allowed_lateness, purge, s->o_key, s->o_start, s->o_end, s->o_res, s->d_st)
        GW_AGG_SWITCH(s->cfg.agg, L);
#undef L
        SCHECK(hipGetLastError());
        if (s->timing) {
            SCHECK(hipEventRecord(ev.second, s->stream));
            s->ev_pending[1].push_back(ev);
        }
        if ((rc = sess_sync(s, err))) return rc;
        if (spec) {
            const bool skipped = s->h_st->overflow || s->h_st->pad[0] || s->h_st->spills;
            if ((rc = sb_finish(s, err))) return rc;
            if (skipped) continue;  // the follow-up has run: fire over the complete state
        }
        s->stats.fires++;
        *fired = (int64_t)s->h_st->rows - before;
        s->wm = wm;
        return GW_OK;
    }
}

void session_rows(SessionState* s, int64_t** k, int64_t** st, int64_t** en, int64_t** r, int64_t* total) {
    *k = s->o_key; *st = s->o_start; *en = s->o_end; *r = s->o_res;
    *total = (int64_t)s->h_st->rows;
}

// Stream-ordered (no host wait): the host view is updated with it, so a refreshed view stays valid.
int session_clear_rows(SessionState* s, std::string& err) { return zero_word_async(s, offsetof(DevStatus, rows), err); }

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
        if ((rc = zero_word_async(s, offsetof(DevStatus, overflow), err))) return rc;  // (the fire's guard)
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
