/*
 * flink_oracle.c — TEST INFRASTRUCTURE ONLY (see flink_oracle.h).
 *
 * CPU restatement of the reference's keyed event-time window path, record by
 * record.  Every function cites the reference code it follows; paths are
 * relative to the Flink tree:
 *   RS/ = flink-runtime/src/main/java/org/apache/flink/streaming/
 *   RR/ = flink-runtime/src/main/java/org/apache/flink/runtime/
 *   C/  = flink-core/src/main/java/org/apache/flink/
 *   SJ/ = flink-streaming-java/src/main/java/org/apache/flink/streaming/
 *
 * Java `long`/`int` arithmetic wraps; it is reproduced with unsigned casts.
 */
#define _POSIX_C_SOURCE 200809L
#include "flink_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define JADD(a, b) ((int64_t)((uint64_t)(a) + (uint64_t)(b)))
#define JSUB(a, b) ((int64_t)((uint64_t)(a) - (uint64_t)(b)))
#define JMUL32(a, b) ((int32_t)((uint32_t)(a) * (uint32_t)(b)))

/* ------------------------------------------------------------------------ */
/* MathUtils (C/util/MathUtils.java)                                          */
/* ------------------------------------------------------------------------ */
static inline int32_t rotl32(int32_t x, int r) {
    uint32_t u = (uint32_t)x;
    return (int32_t)((u << r) | (u >> (32 - r)));
}

/* MathUtils.bitMix, MathUtils.java:194-201 (Murmur3 fmix32). */
int32_t wo_bit_mix(int32_t in) {
    uint32_t h = (uint32_t)in;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return (int32_t)h;
}

/* MathUtils.murmurHash(int), MathUtils.java:137-155. */
int32_t wo_murmur_hash(int32_t code) {
    code = JMUL32(code, 0xcc9e2d51u);
    code = rotl32(code, 15);
    code = JMUL32(code, 0x1b873593u);
    code = rotl32(code, 13);
    code = (int32_t)((uint32_t)JMUL32(code, 5u) + 0xe6546b64u);
    code ^= 4;
    code = wo_bit_mix(code);
    if (code >= 0) return code;
    if (code != INT32_MIN) return -code;
    return 0;
}

/* MathUtils.longToIntWithBitMixing, MathUtils.java:180-185 (TimeWindow.hashCode). */
int32_t wo_long_to_int_with_bit_mixing(int64_t in) {
    uint64_t x = (uint64_t)in;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    x = x ^ (x >> 31);
    return (int32_t)(uint32_t)x;
}

/* JDK Long.hashCode: (int)(value ^ (value >>> 32)). */
int32_t wo_long_hash(int64_t v) {
    uint64_t u = (uint64_t)v;
    return (int32_t)(uint32_t)(u ^ (u >> 32));
}

/* JDK String.hashCode: s[0]*31^(n-1) + ... + s[n-1], int arithmetic. */
int32_t wo_string_hash(const uint16_t* s, int64_t n) {
    uint32_t h = 0;
    for (int64_t i = 0; i < n; i++) h = 31u * h + s[i];
    return (int32_t)h;
}

/* ------------------------------------------------------------------------ */
/* KeyGroupRangeAssignment (RR/state/KeyGroupRangeAssignment.java)            */
/* ------------------------------------------------------------------------ */
/* computeKeyGroupForKeyHash :75-77 */
int32_t wo_assign_to_key_group(int32_t key_hash, int32_t max_parallelism) {
    return wo_murmur_hash(key_hash) % max_parallelism;
}
/* computeOperatorIndexForKeyGroup :124-127 */
int32_t wo_operator_index_for_key_group(int32_t max_p, int32_t p, int32_t kg) {
    return kg * p / max_p;
}
/* computeKeyGroupRangeForOperatorIndex :93-106 */
void wo_key_group_range(int32_t max_p, int32_t p, int32_t idx, int32_t* start, int32_t* end) {
    *start = (idx * max_p + p - 1) / p;
    *end = ((idx + 1) * max_p - 1) / p;
}
/* MathUtils.roundUpToPowerOfTwo :163-171 */
static int32_t round_up_pow2(int32_t x) {
    uint32_t u = (uint32_t)x - 1u;
    u |= u >> 1; u |= u >> 2; u |= u >> 4; u |= u >> 8; u |= u >> 16;
    return (int32_t)(u + 1u);
}
/* computeDefaultMaxParallelism :137-147 (lower bound 128, upper 1<<15) */
int32_t wo_default_max_parallelism(int32_t p) {
    int32_t v = round_up_pow2(p + p / 2);
    if (v < 128) v = 128;
    if (v > 32768) v = 32768;
    return v;
}

/* ------------------------------------------------------------------------ */
/* TimeWindow / assigners                                                     */
/* ------------------------------------------------------------------------ */
/* TimeWindow.getWindowStartWithOffset, RS/api/windowing/windows/TimeWindow.java:264-272 */
int64_t wo_window_start_with_offset(int64_t ts, int64_t offset, int64_t size) {
    int64_t rem = JSUB(ts, offset) % size;
    if (rem < 0) return JSUB(ts, rem + size);
    return JSUB(ts, rem);
}

int wo_validate(const gw_config* c) {
    if (c->assigner == GW_TUMBLING) {
        /* TumblingEventTimeWindows ctor :55-62: abs(offset) >= size -> IAE */
        int64_t ao = c->offset < 0 ? -c->offset : c->offset;
        if (c->size <= 0 || ao >= c->size) return GW_E_INVALID;
    } else if (c->assigner == GW_SLIDING) {
        /* SlidingEventTimeWindows ctor :57-70 */
        int64_t ao = c->offset < 0 ? -c->offset : c->offset;
        if (c->slide <= 0 || ao >= c->slide || c->size <= 0) return GW_E_INVALID;
        if (c->size / c->slide > 10000000) return GW_E_INVALID;
    } else if (c->assigner == GW_SESSION) {
        /* EventTimeSessionWindows ctor: sessionTimeout <= 0 -> IAE (:52-53) */
        if (c->gap <= 0) return GW_E_INVALID;
    } else if (c->assigner == GW_COUNT_TUMBLING) {
        if (c->size <= 0) return GW_E_INVALID;
    } else if (c->assigner == GW_COUNT_SLIDING) {
        if (c->size <= 0 || c->slide <= 0) return GW_E_INVALID;
    } else {
        return GW_E_INVALID;
    }
    if (c->allowed_lateness < 0) return GW_E_INVALID;
    if (c->agg < GW_COUNT || c->agg > GW_SUM_I32) return GW_E_INVALID;
    if ((c->flags & GW_FLAG_BY_FIELD) && (!(c->agg == GW_MIN_I64 || c->agg == GW_MAX_I64 || c->agg == GW_MIN_F64 ||
                                            c->agg == GW_MAX_F64) ||
                                          !(c->assigner == GW_TUMBLING || c->assigner == GW_SLIDING)))
        return GW_E_INVALID;
    if (c->trigger != GW_EVENT_TIME_TRIGGER && c->trigger != GW_PURGING_EVENT_TIME_TRIGGER)
        return GW_E_INVALID;
    return GW_OK;
}

/* TumblingEventTimeWindows.assignWindows :69-85, SlidingEventTimeWindows.assignWindows
 * :77-90, EventTimeSessionWindows.assignWindows (SJ/api/windowing/assigners/
 * EventTimeSessionWindows.java:61-64).  Order = the reference's list order. */
int wo_assign_windows(const gw_config* c, int64_t ts, int64_t* ws, int64_t* we, int cap) {
    if (ts == INT64_MIN) return GW_E_NO_TIMESTAMP;
    if (c->assigner == GW_TUMBLING) {
        if (cap < 1) return GW_E_INVALID;
        int64_t off = c->offset % c->size; /* (globalOffset + staggerOffset(ALIGNED=0)) % size */
        int64_t s = wo_window_start_with_offset(ts, off, c->size);
        ws[0] = s;
        we[0] = JADD(s, c->size);
        return 1;
    }
    if (c->assigner == GW_SLIDING) {
        int n = 0;
        int64_t last = wo_window_start_with_offset(ts, c->offset, c->slide);
        int64_t lim = JSUB(ts, c->size);
        for (int64_t s = last; s > lim; s = JSUB(s, c->slide)) {
            if (n >= cap) return GW_E_RANGE;
            ws[n] = s;
            we[n] = JADD(s, c->size);
            n++;
        }
        return n;
    }
    if (cap < 1) return GW_E_INVALID;
    ws[0] = ts;
    we[0] = JADD(ts, c->gap);
    return 1;
}

/* TimeWindow.intersects :116-118 (inclusive: touching windows merge) */
static inline int tw_intersects(int64_t s1, int64_t e1, int64_t s2, int64_t e2) {
    return s1 <= e2 && e1 >= s2;
}

/* TimeWindow.mergeWindows :208-254: stable sort by start, sweep, cover. */
int wo_merge_windows(int n, const int64_t* s, const int64_t* e, int32_t* group_of,
                     int64_t* gs, int64_t* ge) {
    int* idx = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
    for (int i = 0; i < n; i++) idx[i] = i;
    for (int i = 1; i < n; i++) { /* insertion sort = stable */
        int v = idx[i], j = i - 1;
        while (j >= 0 && s[idx[j]] > s[v]) { idx[j + 1] = idx[j]; j--; }
        idx[j + 1] = v;
    }
    int g = -1;
    for (int k = 0; k < n; k++) {
        int i = idx[k];
        if (g >= 0 && tw_intersects(gs[g], ge[g], s[i], e[i])) {
            if (s[i] < gs[g]) gs[g] = s[i];
            if (e[i] > ge[g]) ge[g] = e[i];
        } else {
            g++;
            gs[g] = s[i];
            ge[g] = e[i];
        }
        group_of[i] = g;
    }
    free(idx);
    return g + 1;
}

/* ------------------------------------------------------------------------ */
/* open-addressing map: 4 x int64 key -> int64 value                          */
/* ------------------------------------------------------------------------ */
typedef struct { int64_t k[4]; int64_t v; int64_t st; } ment_t; /* st 0 empty 1 full 2 tomb */
typedef struct { ment_t* e; int64_t cap, n, used; } map_t;

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}
static uint64_t hash4(const int64_t* k) {
    uint64_t h = mix64((uint64_t)k[0] + 0x9e3779b97f4a7c15ull);
    h = mix64(h ^ (uint64_t)k[1]);
    h = mix64(h ^ (uint64_t)k[2]);
    return mix64(h ^ (uint64_t)k[3]);
}
static int map_init(map_t* m, int64_t cap) {
    int64_t c = 16;
    while (c < cap) c <<= 1;
    m->e = (ment_t*)calloc((size_t)c, sizeof(ment_t));
    m->cap = c; m->n = 0; m->used = 0;
    return m->e ? 0 : -1;
}
static void map_free(map_t* m) { free(m->e); m->e = NULL; m->cap = m->n = m->used = 0; }
static ment_t* map_find(const map_t* m, const int64_t* k) {
    uint64_t mask = (uint64_t)m->cap - 1, i = hash4(k) & mask;
    for (;;) {
        ment_t* e = &m->e[i];
        if (e->st == 0) return NULL;
        if (e->st == 1 && e->k[0] == k[0] && e->k[1] == k[1] && e->k[2] == k[2] && e->k[3] == k[3])
            return e;
        i = (i + 1) & mask;
    }
}
static int map_grow(map_t* m) {
    map_t nm;
    int64_t nc = m->n * 4 > m->cap ? m->cap * 2 : m->cap;
    if (map_init(&nm, nc) != 0) return -1;
    for (int64_t i = 0; i < m->cap; i++) {
        if (m->e[i].st != 1) continue;
        uint64_t mask = (uint64_t)nm.cap - 1, j = hash4(m->e[i].k) & mask;
        while (nm.e[j].st) j = (j + 1) & mask;
        nm.e[j] = m->e[i];
        nm.n++; nm.used++;
    }
    free(m->e);
    *m = nm;
    return 0;
}
/* Returns the entry (existing or newly inserted with v = dflt); *created set. */
static ment_t* map_upsert(map_t* m, const int64_t* k, int64_t dflt, int* created) {
    ment_t* f = map_find(m, k);
    if (f) { if (created) *created = 0; return f; }
    if ((m->used + 1) * 2 > m->cap) {
        if (map_grow(m) != 0) return NULL;
    }
    uint64_t mask = (uint64_t)m->cap - 1, i = hash4(k) & mask;
    while (m->e[i].st == 1) i = (i + 1) & mask;
    if (m->e[i].st == 0) m->used++;
    ment_t* e = &m->e[i];
    memcpy(e->k, k, sizeof(e->k));
    e->v = dflt; e->st = 1;
    m->n++;
    if (created) *created = 1;
    return e;
}
static int map_del(map_t* m, const int64_t* k) {
    ment_t* f = map_find(m, k);
    if (!f) return 0;
    f->st = 2;
    m->n--;
    return 1;
}

/* ------------------------------------------------------------------------ */
/* accumulators (SumFunction / ComparableAggregator / AggregateFunction)      */
/* ------------------------------------------------------------------------ */
typedef struct { int64_t i; double d; int64_t c; int64_t q; /* minBy/maxBy: the element's arrival number */ } acc_t;

static inline double bits2d(int64_t b) { double d; memcpy(&d, &b, 8); return d; }
static inline int64_t d2bits(double d) { int64_t b; memcpy(&b, &d, 8); return b; }

/* Double.compare (JDK): numeric order, then doubleToLongBits (NaN canonical,
 * largest; -0.0 < 0.0). */
static int java_double_compare(double a, double b) {
    if (a < b) return -1;
    if (a > b) return 1;
    int64_t x = (a != a) ? 0x7ff8000000000000LL : d2bits(a);
    int64_t y = (b != b) ? 0x7ff8000000000000LL : d2bits(b);
    return x == y ? 0 : (x < y ? -1 : 1);
}

/* ReduceFunction.reduce(a, b) for the positional aggregations:
 *  SumAggregator.reduce (RS/api/functions/aggregation/SumAggregator.java:66-76) with
 *  SumFunction.{Long,Int,Double}Sum (SumFunction.java:34-105);
 *  ComparableAggregator.reduce non-By branch (ComparableAggregator.java:83-104) with
 *  Min/MaxComparator (Comparator.java:33-90): c==0 -> take b's field. */
static void reduce_into(acc_t* a, int64_t b, int agg) {
    switch (agg) {
    case GW_SUM_I64: a->i = JADD(a->i, b); break;
    case GW_SUM_I32: a->i = (int32_t)((uint32_t)a->i + (uint32_t)b); break;
    case GW_SUM_F64: a->d = a->d + bits2d(b); break;
    case GW_MIN_I64: a->i = (a->i < b) ? a->i : b; break;
    case GW_MAX_I64: a->i = (a->i > b) ? a->i : b; break;
    case GW_MIN_F64: a->d = (java_double_compare(a->d, bits2d(b)) < 0) ? a->d : bits2d(b); break;
    case GW_MAX_F64: a->d = (java_double_compare(a->d, bits2d(b)) > 0) ? a->d : bits2d(b); break;
    default: break;
    }
}

/* minBy / maxBy: ComparableAggregator.reduce, byAggregate branch (ComparableAggregator.java:
 * 88-95) with MinByComparator / MaxByComparator (Comparator.java): c = isExtremal(v1, v2) is 1
 * when value1's field is strictly smaller (MINBY) / larger (MAXBY), 0 when equal (Long.compareTo
 * / Double.compareTo), else -1; c == 0 -> first ? value1 : value2; c == 1 -> value1, else value2.
 * The state element is (field, arrival number q); WindowedStream.minBy/maxBy :725-771. */
static void by_reduce(acc_t* a, int agg, int first, int64_t v, int64_t q) {
    int cmp;
    if (agg == GW_MIN_F64 || agg == GW_MAX_F64) cmp = java_double_compare(a->d, bits2d(v));
    else cmp = a->i < v ? -1 : (a->i > v ? 1 : 0);
    int c = (agg == GW_MIN_I64 || agg == GW_MIN_F64) ? (cmp < 0 ? 1 : cmp == 0 ? 0 : -1)
                                                      : (cmp > 0 ? 1 : cmp == 0 ? 0 : -1);
    if (c == 1 || (c == 0 && first)) return;
    if (agg == GW_MIN_F64 || agg == GW_MAX_F64) a->d = bits2d(v);
    else a->i = v;
    a->q = q;
}

/* First element of a window: ReducingState stores the value itself
 * (HeapReducingState.java:90-97 ReduceTransformation: previous == null ? value : ...);
 * AggregatingState calls createAccumulator then add (HeapAggregatingState.java:94-102). */
static void acc_first(acc_t* a, int agg, int64_t v) {
    memset(a, 0, sizeof(*a));
    switch (agg) {
    case GW_COUNT: a->c = 1; break;
    case GW_AVG_I64: a->i = v; a->c = 1; break;
    case GW_AVG_F64: a->d = 0.0 + bits2d(v); a->c = 1; break;
    case GW_SUM_I32: a->i = (int32_t)v; break;
    case GW_SUM_F64: case GW_MIN_F64: case GW_MAX_F64: a->d = bits2d(v); break;
    default: a->i = v; break;
    }
}
static void acc_add(acc_t* a, int agg, int64_t v) {
    switch (agg) {
    case GW_COUNT: a->c += 1; break;
    case GW_AVG_I64: a->i = JADD(a->i, v); a->c += 1; break;
    case GW_AVG_F64: a->d = a->d + bits2d(v); a->c += 1; break;
    default: reduce_into(a, v, agg); break;
    }
}
/* AbstractHeapMergingState.mergeState(a, b): AggregateFunction.merge or
 * ReduceFunction.reduce (HeapAggregatingState / HeapReducingState). */
static void acc_merge(acc_t* a, const acc_t* b, int agg) {
    switch (agg) {
    case GW_COUNT: a->c += b->c; break;
    case GW_AVG_I64: a->i = JADD(a->i, b->i); a->c += b->c; break;
    case GW_AVG_F64: a->d = a->d + b->d; a->c += b->c; break;
    case GW_SUM_F64: case GW_MIN_F64: case GW_MAX_F64: reduce_into(a, d2bits(b->d), agg); break;
    default: reduce_into(a, b->i, agg); break;
    }
}
/* getResult (AggregateFunction) / the reduced field (PassThroughWindowFunction). */
static int64_t acc_result_bits(const acc_t* a, int agg) {
    switch (agg) {
    case GW_COUNT: return a->c;
    case GW_AVG_I64: return d2bits((double)a->i / (double)a->c);
    case GW_AVG_F64: return d2bits(a->d / (double)a->c);
    case GW_SUM_F64: case GW_MIN_F64: case GW_MAX_F64: return d2bits(a->d);
    default: return a->i;
    }
}

/* ------------------------------------------------------------------------ */
/* operator state                                                             */
/* ------------------------------------------------------------------------ */
typedef struct { int64_t ts, key, s, e, gen; } tmr_t;
typedef struct { int n, cap; int64_t* w; /* [4*i]: ws, we, ss, se */ } mws_t;

struct wo_op {
    gw_config c;
    int64_t wm;
    int64_t late;
    int64_t merges;
    map_t state;  /* (key, ns_start, ns_end, 0) -> acc index */
    acc_t* accs;
    int64_t nacc, cap_acc;
    int64_t* freel;
    int64_t nfree, cap_free;
    map_t timers; /* (ts, key, s, e) -> generation */
    tmr_t* heap;
    int64_t nheap, cap_heap;
    int64_t gen;
    map_t sets;   /* (key,0,0,0) -> index into msets */
    mws_t* msets;
    int64_t nsets, cap_sets;
    int64_t *ok, *os, *oe, *orr;
    int64_t on, ocap, ohead;
    int64_t *lk, *lt, *lv;  /* late side output (GW_FLAG_LATE_SIDE_OUTPUT): the elements themselves */
    int64_t ln, lcap;
    int64_t cur_seq, nseq;  /* arrival number of the element being processed / of the next one */
    int64_t* oq;            /* rows: the arrival number of the window's element (minBy / maxBy) */
    map_t cmap;   /* count windows: (key,0,0,0) -> index into cws */
    map_t khash;  /* (key,0,0,0) -> key.hashCode() of keys given a hash (wo_set_key_hashes) */
    struct cw_s* cws;
    int64_t ncws, cap_cws;
    char err[256];
};

/* Count-window state of one key: the GlobalWindow's contents (the element list the
 * evicting operator keeps, EvictingWindowOperator's ListState) and the CountTrigger's
 * ReducingState<Long> count (CountTrigger.java:39-40). */
typedef struct cw_s {
    int64_t trig;   /* CountTrigger count since its last FIRE                  */
    int64_t total;  /* elements of this key so far (the row's end ordinal)     */
    int64_t n, cap; /* window contents                                         */
    int64_t* v;
    /* restored tumbling contents (wo_restore): the reduced state of `rest` elements that
     * precede v[] -- the reference keeps the ReducingState's value, not the elements */
    int64_t rest;
    acc_t* acc0;
} cw_t;

static void op_err(wo_op* op, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(op->err, sizeof(op->err), fmt, ap);
    va_end(ap);
}

static int64_t acc_alloc(wo_op* op) {
    if (op->nfree > 0) return op->freel[--op->nfree];
    if (op->nacc == op->cap_acc) {
        int64_t nc = op->cap_acc ? op->cap_acc * 2 : 1024;
        acc_t* na = (acc_t*)realloc(op->accs, sizeof(acc_t) * (size_t)nc);
        if (!na) return -1;
        op->accs = na; op->cap_acc = nc;
    }
    return op->nacc++;
}
static void acc_release(wo_op* op, int64_t i) {
    if (op->nfree == op->cap_free) {
        int64_t nc = op->cap_free ? op->cap_free * 2 : 1024;
        op->freel = (int64_t*)realloc(op->freel, sizeof(int64_t) * (size_t)nc);
        op->cap_free = nc;
    }
    op->freel[op->nfree++] = i;
}

/* --- windowState (HeapReducingState / HeapAggregatingState on the
 *     CopyOnWriteStateMap keyed by (key, namespace)) --- */
static int state_add(wo_op* op, int64_t key, int64_t s, int64_t e, int64_t v) {
    int64_t k[4] = {key, s, e, 0};
    int created = 0;
    ment_t* m = map_upsert(&op->state, k, -1, &created);
    if (!m) return GW_E_OOM;
    const int by = (op->c.flags & GW_FLAG_BY_FIELD) != 0;
    if (created) {
        int64_t a = acc_alloc(op);
        if (a < 0) return GW_E_OOM;
        m = map_find(&op->state, k);
        m->v = a;
        acc_first(&op->accs[a], op->c.agg, v);
        op->accs[a].q = op->cur_seq;
    } else if (by) {
        by_reduce(&op->accs[m->v], op->c.agg, !(op->c.flags & GW_FLAG_BY_LAST), v, op->cur_seq);
    } else {
        acc_add(&op->accs[m->v], op->c.agg, v);
    }
    return GW_OK;
}
static acc_t* state_get(wo_op* op, int64_t key, int64_t s, int64_t e) {
    int64_t k[4] = {key, s, e, 0};
    ment_t* m = map_find(&op->state, k);
    return m ? &op->accs[m->v] : NULL;
}
static void state_clear(wo_op* op, int64_t key, int64_t s, int64_t e) {
    int64_t k[4] = {key, s, e, 0};
    ment_t* m = map_find(&op->state, k);
    if (!m) return;
    acc_release(op, m->v);
    map_del(&op->state, k);
}

/* --- timers: InternalTimerServiceImpl + HeapPriorityQueueSet (dedup set + min-heap
 *     on timestamp; InternalTimerServiceImpl.java:249-264,328-347). --- */
static void heap_push(wo_op* op, tmr_t t) {
    if (op->nheap == op->cap_heap) {
        int64_t nc = op->cap_heap ? op->cap_heap * 2 : 1024;
        op->heap = (tmr_t*)realloc(op->heap, sizeof(tmr_t) * (size_t)nc);
        op->cap_heap = nc;
    }
    int64_t i = op->nheap++;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (op->heap[p].ts <= t.ts) break;
        op->heap[i] = op->heap[p];
        i = p;
    }
    op->heap[i] = t;
}
static tmr_t heap_pop(wo_op* op) {
    tmr_t top = op->heap[0];
    tmr_t last = op->heap[--op->nheap];
    int64_t i = 0, n = op->nheap;
    for (;;) {
        int64_t l = 2 * i + 1, r = l + 1, m = i;
        int64_t mts = last.ts;
        if (l < n && op->heap[l].ts < mts) { m = l; mts = op->heap[l].ts; }
        if (r < n && op->heap[r].ts < mts) { m = r; }
        if (m == i) break;
        op->heap[i] = op->heap[m];
        i = m;
    }
    if (n > 0) op->heap[i] = last;
    return top;
}
static int tmr_register(wo_op* op, int64_t key, int64_t s, int64_t e, int64_t ts) {
    int64_t k[4] = {ts, key, s, e};
    int created = 0;
    ment_t* m = map_upsert(&op->timers, k, 0, &created);
    if (!m) return GW_E_OOM;
    if (!created) return GW_OK; /* HeapPriorityQueueSet.add dedups */
    m->v = ++op->gen;
    tmr_t t = {ts, key, s, e, m->v};
    heap_push(op, t);
    return GW_OK;
}
static void tmr_delete(wo_op* op, int64_t key, int64_t s, int64_t e, int64_t ts) {
    int64_t k[4] = {ts, key, s, e};
    map_del(&op->timers, k); /* lazily skipped when popped */
}

/* WindowOperator.cleanupTime :670-677 (overflow -> Long.MAX_VALUE) */
static int64_t cleanup_time(const wo_op* op, int64_t end) {
    int64_t mx = JSUB(end, 1);
    int64_t ct = JADD(mx, op->c.allowed_lateness);
    return ct >= mx ? ct : INT64_MAX;
}
/* WindowOperator.isWindowLate :609-612 */
static int is_window_late(const wo_op* op, int64_t end) { return cleanup_time(op, end) <= op->wm; }
/* WindowOperator.isElementLate :620-624 */
static int is_element_late(const wo_op* op, int64_t ts) {
    return JADD(ts, op->c.allowed_lateness) <= op->wm;
}
/* WindowOperator.registerCleanupTimer :631-643 / deleteCleanupTimer :650-662 */
static int register_cleanup_timer(wo_op* op, int64_t key, int64_t s, int64_t e) {
    int64_t ct = cleanup_time(op, e);
    if (ct == INT64_MAX) return GW_OK;
    return tmr_register(op, key, s, e, ct);
}
static void delete_cleanup_timer(wo_op* op, int64_t key, int64_t s, int64_t e) {
    int64_t ct = cleanup_time(op, e);
    if (ct == INT64_MAX) return;
    tmr_delete(op, key, s, e, ct);
}

/* EventTimeTrigger (RS/api/windowing/triggers/EventTimeTrigger.java:37-79), optionally
 * wrapped in PurgingTrigger (FIRE -> FIRE_AND_PURGE).  Returns 0 CONTINUE, 1 FIRE,
 * 3 FIRE_AND_PURGE. */
static int trigger_on_element(wo_op* op, int64_t key, int64_t s, int64_t e, int* rc) {
    int64_t mx = JSUB(e, 1);
    *rc = GW_OK;
    if (mx <= op->wm) return op->c.trigger == GW_PURGING_EVENT_TIME_TRIGGER ? 3 : 1;
    *rc = tmr_register(op, key, s, e, mx);
    return 0;
}
static int trigger_on_event_time(wo_op* op, int64_t time, int64_t e) {
    if (time != JSUB(e, 1)) return 0;
    return op->c.trigger == GW_PURGING_EVENT_TIME_TRIGGER ? 3 : 1;
}
static void trigger_clear(wo_op* op, int64_t key, int64_t s, int64_t e) {
    tmr_delete(op, key, s, e, JSUB(e, 1));
}
static int trigger_on_merge(wo_op* op, int64_t key, int64_t s, int64_t e) {
    int64_t mx = JSUB(e, 1);
    if (mx > op->wm) return tmr_register(op, key, s, e, mx);
    return GW_OK;
}

/* WindowOperator.emitWindowContents :575-580 (+ InternalSingleValueWindowFunction /
 * PassThroughWindowFunction): row (key, window, result) at timestamp end-1. */
static int emit(wo_op* op, int64_t key, int64_t s, int64_t e, const acc_t* a) {
    if (op->on == op->ocap) {
        int64_t nc = op->ocap ? op->ocap * 2 : 1024;
        op->ok = (int64_t*)realloc(op->ok, 8 * (size_t)nc);
        op->os = (int64_t*)realloc(op->os, 8 * (size_t)nc);
        op->oe = (int64_t*)realloc(op->oe, 8 * (size_t)nc);
        op->orr = (int64_t*)realloc(op->orr, 8 * (size_t)nc);
        op->oq = (int64_t*)realloc(op->oq, 8 * (size_t)nc);
        if (!op->ok || !op->os || !op->oe || !op->orr || !op->oq) return GW_E_OOM;
        op->ocap = nc;
    }
    op->ok[op->on] = key;
    op->os[op->on] = s;
    op->oe[op->on] = e;
    op->orr[op->on] = acc_result_bits(a, op->c.agg);
    op->oq[op->on] = a->q;
    op->on++;
    return GW_OK;
}

/* --- MergingWindowSet (RS/runtime/operators/windowing/MergingWindowSet.java) --- */
static mws_t* mws_get(wo_op* op, int64_t key, int create) {
    int64_t k[4] = {key, 0, 0, 0};
    ment_t* m = map_find(&op->sets, k);
    if (m) return &op->msets[m->v];
    if (!create) return NULL;
    if (op->nsets == op->cap_sets) {
        int64_t nc = op->cap_sets ? op->cap_sets * 2 : 256;
        op->msets = (mws_t*)realloc(op->msets, sizeof(mws_t) * (size_t)nc);
        op->cap_sets = nc;
    }
    int64_t idx = op->nsets++;
    memset(&op->msets[idx], 0, sizeof(mws_t));
    map_upsert(&op->sets, k, idx, NULL);
    return &op->msets[idx];
}
static int mws_find(const mws_t* m, int64_t s, int64_t e) {
    for (int i = 0; i < m->n; i++)
        if (m->w[4 * i] == s && m->w[4 * i + 1] == e) return i;
    return -1;
}
/* mapping.put (replace or append) */
static void mws_put(mws_t* m, int64_t s, int64_t e, int64_t ss, int64_t se) {
    int i = mws_find(m, s, e);
    if (i < 0) {
        if (m->n == m->cap) {
            m->cap = m->cap ? m->cap * 2 : 4;
            m->w = (int64_t*)realloc(m->w, sizeof(int64_t) * 4 * (size_t)m->cap);
        }
        i = m->n++;
        m->w[4 * i] = s;
        m->w[4 * i + 1] = e;
    }
    m->w[4 * i + 2] = ss;
    m->w[4 * i + 3] = se;
}
/* mapping.remove -> returns 1 and the state window if present */
static int mws_remove(mws_t* m, int64_t s, int64_t e, int64_t* ss, int64_t* se) {
    int i = mws_find(m, s, e);
    if (i < 0) return 0;
    if (ss) { *ss = m->w[4 * i + 2]; *se = m->w[4 * i + 3]; }
    m->n--;
    if (i != m->n) memcpy(&m->w[4 * i], &m->w[4 * m->n], 4 * sizeof(int64_t));
    return 1;
}

/* The merge callback of WindowOperator.processElement (WindowOperator.java:314-366). */
static int merge_function(wo_op* op, int64_t key, int64_t rs, int64_t re,
                          const int64_t* mw, int nmw, int64_t tss, int64_t tse,
                          const int64_t* msw, int nmsw) {
    if (JADD(JSUB(re, 1), op->c.allowed_lateness) <= op->wm) {
        op_err(op, "The end timestamp of an event-time window cannot become earlier than the "
                   "current watermark by merging. Current watermark: %lld window: [%lld,%lld)",
               (long long)op->wm, (long long)rs, (long long)re);
        return GW_E_STATE;
    }
    int rc = trigger_on_merge(op, key, rs, re);
    if (rc) return rc;
    for (int i = 0; i < nmw; i++) {
        trigger_clear(op, key, mw[2 * i], mw[2 * i + 1]);
        delete_cleanup_timer(op, key, mw[2 * i], mw[2 * i + 1]);
    }
    /* AbstractHeapMergingState.mergeNamespaces (RR/state/heap/AbstractHeapMergingState.java:65-91) */
    if (nmsw == 0) return GW_OK;
    acc_t merged;
    int have = 0;
    for (int i = 0; i < nmsw; i++) {
        acc_t* src = state_get(op, key, msw[2 * i], msw[2 * i + 1]);
        if (!src) continue;
        acc_t tmp = *src;
        state_clear(op, key, msw[2 * i], msw[2 * i + 1]);
        if (!have) { merged = tmp; have = 1; }
        else acc_merge(&merged, &tmp, op->c.agg);
        op->merges++;
    }
    if (have) {
        int64_t k[4] = {key, tss, tse, 0};
        int created = 0;
        ment_t* m = map_upsert(&op->state, k, -1, &created);
        if (!m) return GW_E_OOM;
        if (created) {
            int64_t a = acc_alloc(op);
            if (a < 0) return GW_E_OOM;
            m = map_find(&op->state, k);
            m->v = a;
            op->accs[a] = merged;
        } else {
            acc_t t = op->accs[m->v];
            acc_merge(&t, &merged, op->c.agg); /* mergeState(targetState, merged) */
            op->accs[m->v] = t;
        }
    }
    return GW_OK;
}

/* The MergeFunction of MergingWindowSet.addWindow (MergingWindowSet.java:210-214):
 * (mergeResult, mergedWindows, stateWindowResult, mergedStateWindows). */
typedef int (*mws_merge_fn)(void* ctx, int64_t key, int64_t rs, int64_t re, const int64_t* mw, int nmw,
                            int64_t tss, int64_t tse, const int64_t* msw, int nmsw);
static int op_merge_fn(void* ctx, int64_t key, int64_t rs, int64_t re, const int64_t* mw, int nmw,
                       int64_t tss, int64_t tse, const int64_t* msw, int nmsw) {
    return merge_function((wo_op*)ctx, key, rs, re, mw, nmw, tss, tse, msw, nmsw);
}

/* MergingWindowSet.addWindow (MergingWindowSet.java:153-224). */
static int mws_add_window_cb(mws_merge_fn fn, void* ctx, int64_t key, mws_t* m, int64_t ns, int64_t ne,
                             int64_t* rs_out, int64_t* re_out) {
    int n = m->n + 1;
    int64_t* s = (int64_t*)malloc(sizeof(int64_t) * 6 * (size_t)n);
    int64_t* e = s + n;
    int64_t* gs = e + n;
    int64_t* ge = gs + n;
    int32_t* grp = (int32_t*)(ge + n);
    for (int i = 0; i < m->n; i++) { s[i] = m->w[4 * i]; e[i] = m->w[4 * i + 1]; }
    s[m->n] = ns;
    e[m->n] = ne;
    int ng = wo_merge_windows(n, s, e, grp, gs, ge);

    int64_t rs = ns, re = ne;
    int merged_new = 0, any_merge = 0, rc = GW_OK;
    int64_t* mw = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)n);
    int64_t* msw = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)n);
    for (int g = 0; g < ng && rc == GW_OK; g++) {
        /* members as a Set (duplicates collapse, TimeWindow.mergeWindows builds a HashSet) */
        int nm = 0;
        int has_new = 0;
        for (int i = 0; i < n; i++) {
            if (grp[i] != g) continue;
            int dup = 0;
            for (int j = 0; j < nm; j++)
                if (mw[2 * j] == s[i] && mw[2 * j + 1] == e[i]) dup = 1;
            if (dup) continue;
            mw[2 * nm] = s[i];
            mw[2 * nm + 1] = e[i];
            nm++;
        }
        if (nm <= 1) continue; /* mergeWindows only calls back for size > 1 */
        any_merge = 1;
        /* mergedWindows.remove(newWindow) */
        for (int j = 0; j < nm; j++) {
            if (mw[2 * j] == ns && mw[2 * j + 1] == ne) {
                has_new = 1;
                memmove(&mw[2 * j], &mw[2 * j + 2], sizeof(int64_t) * 2 * (size_t)(nm - j - 1));
                nm--;
                break;
            }
        }
        if (has_new) { merged_new = 1; rs = gs[g]; re = ge[g]; }
        /* mergedStateWindow = mapping.get(mergedWindows.iterator().next()) */
        int fi = mws_find(m, mw[0], mw[1]);
        int64_t tss = m->w[4 * fi + 2], tse = m->w[4 * fi + 3];
        int nmsw = 0;
        for (int j = 0; j < nm; j++) {
            int64_t a, b;
            if (mws_remove(m, mw[2 * j], mw[2 * j + 1], &a, &b)) {
                msw[2 * nmsw] = a;
                msw[2 * nmsw + 1] = b;
                nmsw++;
            }
        }
        mws_put(m, gs[g], ge[g], tss, tse);
        for (int j = 0; j < nmsw; j++) { /* mergedStateWindows.remove(mergedStateWindow) */
            if (msw[2 * j] == tss && msw[2 * j + 1] == tse) {
                memmove(&msw[2 * j], &msw[2 * j + 2], sizeof(int64_t) * 2 * (size_t)(nmsw - j - 1));
                nmsw--;
                break;
            }
        }
        int contains_result = 0;
        for (int j = 0; j < nm; j++)
            if (mw[2 * j] == gs[g] && mw[2 * j + 1] == ge[g]) contains_result = 1;
        if (!(contains_result && nm == 1))
            rc = fn(ctx, key, gs[g], ge[g], mw, nm, tss, tse, msw, nmsw);
    }
    if (rc == GW_OK && (!any_merge || (rs == ns && re == ne && !merged_new)))
        mws_put(m, rs, re, rs, re);
    free(mw);
    free(msw);
    free(s);
    *rs_out = rs;
    *re_out = re;
    return rc;
}
static int mws_add_window(wo_op* op, int64_t key, mws_t* m, int64_t ns, int64_t ne,
                          int64_t* rs_out, int64_t* re_out) {
    return mws_add_window_cb(op_merge_fn, op, key, m, ns, ne, rs_out, re_out);
}

/* A stand-alone MergingWindowSet of EventTimeSessionWindows (test hook for the reference's
 * MergingWindowSetTest, SJT/runtime/operators/windowing/MergingWindowSetTest.java:62-495):
 * addWindow with a recording MergeFunction, getStateWindow, retireWindow, the restore from
 * a ListState and the persisted list. */
struct wo_mws {
    mws_t m;
    int merged;                   /* the MergeFunction ran during the last add */
    int64_t target[2], state[2];  /* mergeResult, stateWindowResult */
    int nsrc, nmsw;
    int64_t src[2 * 64], msw[2 * 64];
};
static int rec_merge_fn(void* ctx, int64_t key, int64_t rs, int64_t re, const int64_t* mw, int nmw,
                        int64_t tss, int64_t tse, const int64_t* msw, int nmsw) {
    (void)key;
    wo_mws* w = (wo_mws*)ctx;
    if (w->merged) return GW_E_STATE; /* "More than one merge for adding a Window should not occur." */
    if (nmw > 64 || nmsw > 64) return GW_E_UNSUPPORTED;
    w->merged = 1;
    w->target[0] = rs; w->target[1] = re;
    w->state[0] = tss; w->state[1] = tse;
    w->nsrc = nmw;
    memcpy(w->src, mw, sizeof(int64_t) * 2 * (size_t)nmw);
    w->nmsw = nmsw;
    memcpy(w->msw, msw, sizeof(int64_t) * 2 * (size_t)nmsw);
    return GW_OK;
}
wo_mws* wo_mws_create(void) { return (wo_mws*)calloc(1, sizeof(wo_mws)); }
void wo_mws_destroy(wo_mws* w) {
    if (!w) return;
    free(w->m.w);
    free(w);
}
/* addWindow(new TimeWindow(s, e), mergeFunction): result window into res[2]; info[] gets
 * merged, target (2), state window (2), nsrc, nsrc x (s, e), nmsw, nmsw x (s, e). */
int wo_mws_add(wo_mws* w, int64_t s, int64_t e, int64_t* res, int64_t* info) {
    w->merged = 0;
    w->nsrc = w->nmsw = 0;
    int rc = mws_add_window_cb(rec_merge_fn, w, 0, &w->m, s, e, &res[0], &res[1]);
    if (rc) return rc;
    int q = 0;
    info[q++] = w->merged;
    info[q++] = w->target[0]; info[q++] = w->target[1];
    info[q++] = w->state[0]; info[q++] = w->state[1];
    info[q++] = w->nsrc;
    for (int i = 0; i < 2 * w->nsrc; i++) info[q++] = w->src[i];
    info[q++] = w->nmsw;
    for (int i = 0; i < 2 * w->nmsw; i++) info[q++] = w->msw[i];
    return GW_OK;
}
/* getStateWindow: 1 and the state window in out[2], 0 when the window is not in flight */
int wo_mws_state_window(const wo_mws* w, int64_t s, int64_t e, int64_t* out) {
    int i = mws_find(&w->m, s, e);
    if (i < 0) return 0;
    out[0] = w->m.w[4 * i + 2];
    out[1] = w->m.w[4 * i + 3];
    return 1;
}
/* retireWindow: GW_E_STATE ("not in in-flight window set") when absent */
int wo_mws_retire(wo_mws* w, int64_t s, int64_t e) {
    return mws_remove(&w->m, s, e, NULL, NULL) ? GW_OK : GW_E_STATE;
}
/* the constructor's restore from the ListState: mapping.put(f0, f1) per element */
void wo_mws_put(wo_mws* w, int64_t s, int64_t e, int64_t ss, int64_t se) { mws_put(&w->m, s, e, ss, se); }
/* persist(): the mapping as (window, state window) quadruples; returns their number */
int wo_mws_list(const wo_mws* w, int64_t* out, int cap) {
    for (int i = 0; i < w->m.n && i < cap; i++) memcpy(out + 4 * i, w->m.w + 4 * i, 4 * sizeof(int64_t));
    return w->m.n;
}

/* ------------------------------------------------------------------------ */
/* WindowOperator.processElement (WindowOperator.java:293-447)                */
/* ------------------------------------------------------------------------ */
/* Count windows, element by element (GlobalWindows.assignWindows -> the single
 * GlobalWindow, RS/api/windowing/assigners/GlobalWindows.java:50-53):
 *  - countWindow(size) = PurgingTrigger(CountTrigger(size)) (KeyedStream.java:676-678):
 *    the element joins the window state; CountTrigger.onElement (CountTrigger.java:47-56)
 *    counts it and FIREs at count >= size, clearing its count; PurgingTrigger turns FIRE
 *    into FIRE_AND_PURGE, so the window state is emitted and cleared
 *    (WindowOperator.processElement :408-446, PurgingTrigger.onElement :44-48);
 *  - countWindow(size, slide) = CountEvictor(size) + CountTrigger(slide)
 *    (KeyedStream.java:686-690): on FIRE the evicting operator runs
 *    CountEvictor.evictBefore, which drops the oldest elements beyond `size`
 *    (CountEvictor.java:50-85), and emits the function over the rest
 *    (EvictingWindowOperator.emitWindowContents :373-410); nothing is purged.
 * The function folds the contents in arrival order (ReduceApplyWindowFunction /
 * AggregateApplyWindowFunction), as acc_first/acc_add do.  GlobalWindows is not an
 * event-time assigner, so nothing is ever late and MAX_WATERMARK fires nothing. */
static int count_process_element(wo_op* op, int64_t key, int64_t v) {
    int64_t k[4] = {key, 0, 0, 0};
    int created = 0;
    ment_t* m = map_upsert(&op->cmap, k, op->ncws, &created);
    if (!m) { op_err(op, "out of memory"); return GW_E_OOM; }
    if (created) {
        if (op->ncws == op->cap_cws) {
            int64_t nc = op->cap_cws ? op->cap_cws * 2 : 1024;
            cw_t* nw = (cw_t*)realloc(op->cws, sizeof(cw_t) * (size_t)nc);
            if (!nw) { op_err(op, "out of memory"); return GW_E_OOM; }
            op->cws = nw;
            op->cap_cws = nc;
        }
        memset(&op->cws[op->ncws], 0, sizeof(cw_t));
        op->ncws++;
    }
    cw_t* w = &op->cws[m->v];
    if (w->n == w->cap) {
        int64_t nc = w->cap ? w->cap * 2 : 16;
        int64_t* nv = (int64_t*)realloc(w->v, 8 * (size_t)nc);
        if (!nv) { op_err(op, "out of memory"); return GW_E_OOM; }
        w->v = nv;
        w->cap = nc;
    }
    w->v[w->n++] = v;
    w->total++;
    const int sliding = op->c.assigner == GW_COUNT_SLIDING;
    const int64_t max_count = sliding ? op->c.slide : op->c.size;
    if (++w->trig < max_count) return GW_OK;
    w->trig = 0; /* CountTrigger: count.clear() before FIRE */
    if (sliding && w->n > op->c.size) {
        int64_t drop = w->n - op->c.size;
        memmove(w->v, w->v + drop, 8 * (size_t)(w->n - drop));
        w->n -= drop;
    }
    acc_t a;
    int64_t i0 = 0;
    if (w->acc0) { /* restored contents first (tumbling only) */
        a = *w->acc0;
    } else {
        acc_first(&a, op->c.agg, w->v[0]);
        i0 = 1;
    }
    for (int64_t i = i0; i < w->n; i++) acc_add(&a, op->c.agg, w->v[i]);
    int rc = emit(op, key, w->total - w->n - w->rest, w->total, &a);
    if (!sliding) { /* FIRE_AND_PURGE */
        w->n = 0;
        w->rest = 0;
        free(w->acc0);
        w->acc0 = NULL;
    }
    return rc;
}

int wo_process_element(wo_op* op, int64_t key, int64_t ts, int64_t v) {
    op->cur_seq = op->nseq++;
    if (op->c.assigner == GW_COUNT_TUMBLING || op->c.assigner == GW_COUNT_SLIDING)
        return count_process_element(op, key, v);
    int64_t ws[64], we[64];
    int64_t* pws = ws;
    int64_t* pwe = we;
    int cap = 64;
    if (op->c.assigner == GW_SLIDING) {
        int64_t need = op->c.size / op->c.slide + 2;
        if (need > cap) {
            pws = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)need);
            pwe = pws + need;
            cap = (int)need;
        }
    }
    int nw = wo_assign_windows(&op->c, ts, pws, pwe, cap);
    int rc = GW_OK;
    if (nw < 0) {
        op_err(op, "Record has Long.MIN_VALUE timestamp (= no timestamp marker).");
        rc = nw;
        goto out;
    }
    int skipped = 1;
    if (op->c.assigner == GW_SESSION) {
        mws_t* m = mws_get(op, key, 1);
        for (int w = 0; w < nw && rc == GW_OK; w++) {
            int64_t as, ae;
            rc = mws_add_window(op, key, m, pws[w], pwe[w], &as, &ae);
            if (rc) break;
            if (is_window_late(op, ae)) {
                mws_remove(m, as, ae, NULL, NULL); /* retireWindow */
                continue;
            }
            skipped = 0;
            int i = mws_find(m, as, ae);
            if (i < 0) { op_err(op, "Window is not in in-flight window set."); rc = GW_E_STATE; break; }
            int64_t ss = m->w[4 * i + 2], se = m->w[4 * i + 3];
            rc = state_add(op, key, ss, se, v);
            if (rc) break;
            int r = trigger_on_element(op, key, as, ae, &rc);
            if (rc) break;
            if (r & 1) {
                acc_t* a = state_get(op, key, ss, se);
                if (a) rc = emit(op, key, as, ae, a);
            }
            if (r & 2) state_clear(op, key, ss, se);
            if (rc == GW_OK) rc = register_cleanup_timer(op, key, as, ae);
        }
    } else {
        for (int w = 0; w < nw && rc == GW_OK; w++) {
            if (is_window_late(op, pwe[w])) continue;
            skipped = 0;
            rc = state_add(op, key, pws[w], pwe[w], v);
            if (rc) break;
            int r = trigger_on_element(op, key, pws[w], pwe[w], &rc);
            if (rc) break;
            if (r & 1) {
                acc_t* a = state_get(op, key, pws[w], pwe[w]);
                if (a) rc = emit(op, key, pws[w], pwe[w], a);
            }
            if (r & 2) state_clear(op, key, pws[w], pwe[w]);
            if (rc == GW_OK) rc = register_cleanup_timer(op, key, pws[w], pwe[w]);
        }
    }
    /* WindowOperator.java:440-446: a skipped late element goes to the late-data side output
     * when one is set (sideOutput :587-588), else it is counted in numLateRecordsDropped */
    if (rc == GW_OK && skipped && is_element_late(op, ts)) {
        if (op->c.flags & GW_FLAG_LATE_SIDE_OUTPUT) {
            if (op->ln == op->lcap) {
                int64_t nc = op->lcap ? op->lcap * 2 : 256;
                op->lk = (int64_t*)realloc(op->lk, 8 * (size_t)nc);
                op->lt = (int64_t*)realloc(op->lt, 8 * (size_t)nc);
                op->lv = (int64_t*)realloc(op->lv, 8 * (size_t)nc);
                op->lcap = nc;
            }
            op->lk[op->ln] = key; op->lt[op->ln] = ts; op->lv[op->ln] = v;
            op->ln++;
        } else {
            op->late++;
        }
    }
out:
    if (pws != ws) free(pws);
    return rc;
}

int wo_process_batch(wo_op* op, int64_t n, const int64_t* key, const int64_t* ts,
                     const int64_t* v) {
    for (int64_t i = 0; i < n; i++) {
        int rc = wo_process_element(op, key[i], ts[i], v ? v[i] : 0);
        if (rc) return rc;
    }
    return GW_OK;
}

/* WindowOperator.onEventTime (WindowOperator.java:450-494) + clearAllState :560-571 */
static int on_event_time(wo_op* op, const tmr_t* t) {
    int64_t ns_s, ns_e;
    mws_t* m = NULL;
    if (op->c.assigner == GW_SESSION) {
        m = mws_get(op, t->key, 0);
        int i = m ? mws_find(m, t->s, t->e) : -1;
        if (i < 0) return GW_OK; /* timer for a non-existent window */
        ns_s = m->w[4 * i + 2];
        ns_e = m->w[4 * i + 3];
    } else {
        ns_s = t->s;
        ns_e = t->e;
    }
    int r = trigger_on_event_time(op, t->ts, t->e);
    int rc = GW_OK;
    if (r & 1) {
        acc_t* a = state_get(op, t->key, ns_s, ns_e);
        if (a) rc = emit(op, t->key, t->s, t->e, a);
    }
    if (r & 2) state_clear(op, t->key, ns_s, ns_e);
    if (t->ts == cleanup_time(op, t->e)) { /* isCleanupTime */
        state_clear(op, t->key, ns_s, ns_e);
        trigger_clear(op, t->key, t->s, t->e);
        if (m) mws_remove(m, t->s, t->e, NULL, NULL);
    }
    return rc;
}

/* AbstractStreamOperator.processWatermark -> InternalTimerServiceImpl.tryAdvanceWatermark
 * (InternalTimerServiceImpl.java:328-347): currentWatermark = wm, then poll every
 * timer with timestamp <= wm. */
int wo_process_watermark(wo_op* op, int64_t wm) {
    if (wm <= op->wm) return GW_OK;
    op->wm = wm;
    while (op->nheap > 0 && op->heap[0].ts <= wm) {
        tmr_t t = heap_pop(op);
        int64_t k[4] = {t.ts, t.key, t.s, t.e};
        ment_t* m = map_find(&op->timers, k);
        if (!m || m->v != t.gen) continue; /* deleted (or re-registered later) */
        map_del(&op->timers, k);
        int rc = on_event_time(op, &t);
        if (rc) return rc;
    }
    return GW_OK;
}

/* ------------------------------------------------------------------------ */
wo_op* wo_create(const gw_config* cfg) {
    if (wo_validate(cfg) != GW_OK) return NULL;
    wo_op* op = (wo_op*)calloc(1, sizeof(wo_op));
    if (!op) return NULL;
    op->c = *cfg;
    op->wm = INT64_MIN;
    if (map_init(&op->state, 1024) || map_init(&op->timers, 1024) || map_init(&op->sets, 256) ||
        map_init(&op->cmap, 1024) || map_init(&op->khash, 64)) {
        wo_destroy(op);
        return NULL;
    }
    return op;
}

void wo_destroy(wo_op* op) {
    if (!op) return;
    map_free(&op->state);
    map_free(&op->timers);
    map_free(&op->sets);
    map_free(&op->cmap);
    map_free(&op->khash);
    for (int64_t i = 0; i < op->ncws; i++) { free(op->cws[i].v); free(op->cws[i].acc0); }
    free(op->cws);
    for (int64_t i = 0; i < op->nsets; i++) free(op->msets[i].w);
    free(op->msets);
    free(op->accs);
    free(op->freel);
    free(op->heap);
    free(op->ok); free(op->os); free(op->oe); free(op->orr); free(op->oq);
    free(op->lk); free(op->lt); free(op->lv);
    free(op);
}

int64_t wo_late_output_count(const wo_op* op) { return op->ln; }
int64_t wo_drain_late(wo_op* op, int64_t* key, int64_t* ts, int64_t* v, int64_t cap) {
    int64_t n = op->ln < cap ? op->ln : cap;
    for (int64_t i = 0; i < n; i++) { key[i] = op->lk[i]; ts[i] = op->lt[i]; v[i] = op->lv[i]; }
    memmove(op->lk, op->lk + n, 8 * (size_t)(op->ln - n));
    memmove(op->lt, op->lt + n, 8 * (size_t)(op->ln - n));
    memmove(op->lv, op->lv + n, 8 * (size_t)(op->ln - n));
    op->ln -= n;
    return n;
}

int64_t wo_output_count(const wo_op* op) { return op->on - op->ohead; }

int64_t wo_drain(wo_op* op, int64_t* key, int64_t* s, int64_t* e, int64_t* r, int64_t cap) {
    return wo_drain_seq(op, key, s, e, r, NULL, cap);
}

int64_t wo_drain_seq(wo_op* op, int64_t* key, int64_t* s, int64_t* e, int64_t* r, int64_t* q, int64_t cap) {
    int64_t n = op->on - op->ohead;
    if (n > cap) n = cap;
    for (int64_t i = 0; i < n; i++) {
        int64_t j = op->ohead + i;
        if (key) key[i] = op->ok[j];
        if (s) s[i] = op->os[j];
        if (e) e[i] = op->oe[j];
        if (r) r[i] = op->orr[j];
        if (q) q[i] = op->oq[j];
    }
    op->ohead += n;
    if (op->ohead == op->on) op->ohead = op->on = 0;
    return n;
}

int64_t wo_late_dropped(const wo_op* op) { return op->late; }
void wo_set_arrival(wo_op* op, int64_t next) { op->nseq = next; }
int64_t wo_current_watermark(const wo_op* op) { return op->wm; }
int64_t wo_state_entries(const wo_op* op) { return op->state.n; }
int64_t wo_timer_count(const wo_op* op) { return op->timers.n; }
int64_t wo_session_merges(const wo_op* op) { return op->merges; }
const char* wo_last_error(const wo_op* op) { return op ? op->err : "null operator"; }

/* ------------------------------------------------------------------------ */
/* Snapshot / restore in the heap backend's per-key-group layout              */
/* ------------------------------------------------------------------------ */
/* The keyed state of the reference's WindowOperator is written per key group
 * (HeapSnapshotStrategy.java:97-154): for each registered state its
 * CopyOnWriteStateMapSnapshot.writeState (:127-149) -- int n, then n x (namespace, key,
 * state), each with its serializer (big-endian DataOutputView) -- and the event-time
 * timers of the key group (InternalTimerServiceImpl.snapshotTimersForKeyGroup :350-360),
 * each as TimerSerializer.serialize writes it (:147-152: flipSignBit(timestamp), key,
 * namespace).  The blob (version 4, include/gpuwin.h gw_snapshot) carries per key group:
 *   "window-contents":    int32 n; n x (window.start, window.end, key, accumulator)
 *                         (TimeWindow.Serializer :159-169, LongSerializer, and the
 *                         accumulator as LongSerializer / DoubleSerializer / IntSerializer /
 *                         Tuple2(sum, count) for the closed set of aggregates);
 *   "merging-window-set": int32 m; m x (key, [int32 key hash,] int32 c, c x (window, state window)) -- the
 *                         MergingWindowSet ListState<Tuple2<W, W>> of session windows
 *                         (MergingWindowSet.persist :99-106); 0 for other assigners;
 *   timers:               int32 t; t x (flipSignBit(ts), key, window.start, window.end).
 * The watermark is not state: after a restore it is Long.MIN_VALUE
 * (InternalTimerServiceImpl.java:72), so nothing restored is late until the next
 * watermark. */
typedef struct { uint8_t* p; int64_t n, cap; } wbuf;
static void wb_put(wbuf* b, const void* src, int64_t n) {
    if (b->p && b->n + n <= b->cap) memcpy(b->p + b->n, src, (size_t)n);
    b->n += n;
}
static void wb_be64(wbuf* b, int64_t v) {
    uint8_t x[8];
    for (int i = 0; i < 8; i++) x[i] = (uint8_t)((uint64_t)v >> (56 - 8 * i));
    wb_put(b, x, 8);
}
static void wb_be32(wbuf* b, int32_t v) {
    uint8_t x[4];
    for (int i = 0; i < 4; i++) x[i] = (uint8_t)((uint32_t)v >> (24 - 8 * i));
    wb_put(b, x, 4);
}
static int64_t rd_be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    return (int64_t)v;
}
static int32_t rd_be32(const uint8_t* p) {
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) v = (v << 8) | p[i];
    return (int32_t)v;
}
static void wb_acc(wbuf* b, int agg, const acc_t* a) {
    switch (agg) {
    case GW_COUNT: wb_be64(b, a->c); break;
    case GW_SUM_I32: wb_be32(b, (int32_t)a->i); break;
    case GW_SUM_F64: case GW_MIN_F64: case GW_MAX_F64: wb_be64(b, d2bits(a->d)); break;
    case GW_AVG_I64: wb_be64(b, a->i); wb_be64(b, a->c); break;
    case GW_AVG_F64: wb_be64(b, d2bits(a->d)); wb_be64(b, a->c); break;
    default: wb_be64(b, a->i); break;
    }
}
int wo_acc_bytes(int agg) {
    return agg == GW_SUM_I32 ? 4 : (agg == GW_AVG_I64 || agg == GW_AVG_F64) ? 16 : 8;
}
static void rd_acc(const uint8_t* p, int agg, acc_t* a) {
    memset(a, 0, sizeof(*a));
    switch (agg) {
    case GW_COUNT: a->c = rd_be64(p); break;
    case GW_SUM_I32: a->i = rd_be32(p); break;
    case GW_SUM_F64: case GW_MIN_F64: case GW_MAX_F64: a->d = bits2d(rd_be64(p)); break;
    case GW_AVG_I64: a->i = rd_be64(p); a->c = rd_be64(p + 8); break;
    case GW_AVG_F64: a->d = bits2d(rd_be64(p)); a->c = rd_be64(p + 8); break;
    default: a->i = rd_be64(p); break;
    }
}

typedef struct { int32_t kg; int64_t k0, k1, k2, k3; int64_t v; } snap_ent;
static int cmp_snap_ent(const void* a, const void* b) {
    const snap_ent* x = (const snap_ent*)a;
    const snap_ent* y = (const snap_ent*)b;
    if (x->kg != y->kg) return x->kg < y->kg ? -1 : 1;
    const int64_t xs[4] = {x->k0, x->k1, x->k2, x->k3}, ys[4] = {y->k0, y->k1, y->k2, y->k3};
    for (int i = 0; i < 4; i++)
        if (xs[i] != ys[i]) return xs[i] < ys[i] ? -1 : 1;
    return 0;
}
/* The key's Java hashCode: the one given with wo_set_key_hashes (the caller's key ids stand
 * for String / Integer / ... keys), else Long.hashCode. */
static int32_t key_hash_of(const wo_op* op, int64_t key) {
    if (op->khash.n) {
        const int64_t k[4] = {key, 0, 0, 0};
        const ment_t* m = map_find(&op->khash, k);
        if (m) return (int32_t)m->v;
    }
    return wo_long_hash(key);
}
static int32_t key_group_of(const wo_op* op, int64_t key) {
    return wo_assign_to_key_group(key_hash_of(op, key), op->c.max_parallelism > 0 ? op->c.max_parallelism : 128);
}

int wo_set_key_hashes(wo_op* op, int64_t n, const int64_t* key, const int32_t* hash) {
    for (int64_t i = 0; i < n; i++) {
        const int64_t k[4] = {key[i], 0, 0, 0};
        int created = 0;
        ment_t* m = map_upsert(&op->khash, k, hash[i], &created);
        if (!m) return GW_E_OOM;
        if (!created && m->v != hash[i]) { op_err(op, "a key with two different key hashes"); return GW_E_INVALID; }
    }
    return GW_OK;
}

/* The 96-byte blob header (include/gpuwin.h gw_snapshot, gw_runtime.cpp SnapHeader). */
static void snap_header(const wo_op* op, int32_t kg_lo, int32_t kg_hi, int hashed, int64_t payload, uint8_t* h) {
    memset(h, 0, 96);
    memcpy(h, "GWS1", 4);
    const uint32_t ver = 4;
    const int64_t slide = op->c.assigner == GW_TUMBLING ? op->c.size : op->c.slide;
    const int32_t i32s[2] = {op->c.agg, op->c.assigner};
    const int64_t i64s[5] = {op->c.size, slide, op->c.offset, op->c.gap,
                             (hashed ? 1 : 0) | ((op->c.flags & GW_FLAG_BY_FIELD) ? 2 : 0)};
    const int32_t mp = op->c.max_parallelism > 0 ? op->c.max_parallelism : 128;
    const int32_t i32b[4] = {mp, kg_lo, kg_hi, 0};
    const int64_t tail[3] = {0, 0, payload};
    memcpy(h + 4, &ver, 4);
    memcpy(h + 8, i32s, 8);
    memcpy(h + 16, i64s, 40);
    memcpy(h + 56, i32b, 16);
    memcpy(h + 72, tail, 24);
}

/* countWindow(size) = GlobalWindows + PurgingTrigger(CountTrigger(size)) (KeyedStream.java:
 * 676-678) in the heap layout, per key group:
 *   "window-contents": int32 n; n x (GlobalWindow, key, [int32 key hash,] state): the reduced
 *                      contents since the key's last FIRE_AND_PURGE (GlobalWindow.Serializer
 *                      writes one byte 0, GlobalWindow.java:96-98);
 *   "count":           int32 m; m x (GlobalWindow, key, [int32 key hash,] long): CountTrigger's
 *                      ReducingState<Long> "count" (CountTrigger.java:39-40, cleared at each
 *                      FIRE :52-55);
 *   timers:            int32 0 -- GlobalWindows is not an event-time assigner and its window
 *                      ends at Long.MAX_VALUE, so no cleanup timer (WindowOperator.java:631-643)
 *                      and CountTrigger registers none.
 * A key right after a FIRE_AND_PURGE holds no state.  Keys ascending within a key group.  The
 * sliding form (CountEvictor + CountTrigger(slide)) keeps the element list itself and is not
 * written here. */
static int64_t count_snapshot(wo_op* op, int32_t kg_lo, int32_t kg_hi, uint8_t* buf, int64_t cap) {
    if (op->c.assigner != GW_COUNT_TUMBLING) return GW_E_UNSUPPORTED;
    if (kg_lo < 0 || kg_hi < kg_lo) return GW_E_INVALID;
    const int nk = kg_hi - kg_lo + 1;
    const int hashed = op->khash.n > 0;
    int64_t ne = 0;
    snap_ent* se = (snap_ent*)malloc(sizeof(snap_ent) * (size_t)(op->ncws + 1));
    if (!se) return GW_E_OOM;
    for (int64_t i = 0; i < op->cmap.cap; i++) {
        const ment_t* m = &op->cmap.e[i];
        if (m->st != 1 || op->cws[m->v].trig == 0) continue;
        const int32_t kg = key_group_of(op, m->k[0]);
        if (kg < kg_lo || kg > kg_hi) continue;
        se[ne++] = (snap_ent){kg, m->k[0], 0, 0, 0, m->v};
    }
    qsort(se, (size_t)ne, sizeof(snap_ent), cmp_snap_ent);
    const int64_t pay0 = 96 + (int64_t)(nk + 1) * 8;
    wbuf b = {buf, pay0, cap};
    int64_t* offs = (int64_t*)calloc((size_t)nk + 1, sizeof(int64_t));
    const uint8_t global_window = 0;
    int64_t a = 0;
    for (int g = 0; g < nk; g++) {
        const int32_t kg = kg_lo + g;
        offs[g] = b.n - pay0;
        int64_t a1 = a;
        while (a1 < ne && se[a1].kg == kg) a1++;
        wb_be32(&b, (int32_t)(a1 - a));
        for (int64_t q = a; q < a1; q++) {
            const cw_t* w = &op->cws[se[q].v];
            acc_t acc;
            int64_t i0 = 0;
            if (w->acc0) {
                acc = *w->acc0;
            } else {
                acc_first(&acc, op->c.agg, w->v[0]);
                i0 = 1;
            }
            for (int64_t i = i0; i < w->n; i++) acc_add(&acc, op->c.agg, w->v[i]);
            wb_put(&b, &global_window, 1);
            wb_be64(&b, se[q].k0);
            if (hashed) wb_be32(&b, key_hash_of(op, se[q].k0));
            wb_acc(&b, op->c.agg, &acc);
        }
        wb_be32(&b, (int32_t)(a1 - a));
        for (int64_t q = a; q < a1; q++) {
            wb_put(&b, &global_window, 1);
            wb_be64(&b, se[q].k0);
            if (hashed) wb_be32(&b, key_hash_of(op, se[q].k0));
            wb_be64(&b, op->cws[se[q].v].trig);
        }
        wb_be32(&b, 0);
        a = a1;
    }
    offs[nk] = b.n - pay0;
    const int64_t total = b.n;
    if (buf && cap >= total) {
        snap_header(op, kg_lo, kg_hi, hashed, offs[nk], buf);
        memcpy(buf + 96, offs, (size_t)(nk + 1) * 8);
    }
    free(offs);
    free(se);
    return total;
}

/* The restore side of count_snapshot: every (key, contents) entry pairs with the key's
 * CountTrigger count (a count without contents, or contents without a count, is a state
 * this operator never writes: GW_E_INVALID). */
static int count_restore(wo_op* op, const uint8_t* p, const uint8_t* end, int nk, int hb) {
    const int ab = wo_acc_bytes(op->c.agg);
#define NEED(x) do { if ((int64_t)(x) > end - p) { op_err(op, "truncated snapshot blob"); return GW_E_INVALID; } } while (0)
    for (int g = 0; g < nk; g++) {
        NEED(4);
        const int32_t n = rd_be32(p); p += 4;
        if (n < 0) { op_err(op, "corrupt snapshot blob"); return GW_E_INVALID; }
        NEED((int64_t)n * (9 + hb + ab));
        const uint8_t* st = p;
        p += (int64_t)n * (9 + hb + ab);
        NEED(4);
        const int32_t m = rd_be32(p); p += 4;
        if (m != n) { op_err(op, "count-window contents without their CountTrigger count"); return GW_E_INVALID; }
        NEED((int64_t)m * (17 + hb));
        for (int32_t i = 0; i < n; i++) {
            const uint8_t* x = st + (int64_t)i * (9 + hb + ab);
            const uint8_t* c = p + (int64_t)i * (17 + hb);
            int64_t key = rd_be64(x + 1);
            const int64_t cnt = rd_be64(c + 9 + hb);
            if (x[0] != 0 || c[0] != 0 || rd_be64(c + 1) != key || cnt <= 0 || cnt >= op->c.size) {
                op_err(op, "corrupt count-window snapshot entry");
                return GW_E_INVALID;
            }
            if (hb) {
                const int32_t kh = rd_be32(x + 9);
                const int rc = wo_set_key_hashes(op, 1, &key, &kh);
                if (rc) return rc;
            }
            const int64_t k[4] = {key, 0, 0, 0};
            int created = 0;
            ment_t* me = map_upsert(&op->cmap, k, op->ncws, &created);
            if (!me) return GW_E_OOM;
            if (!created) { op_err(op, "a restored key already holds count-window state"); return GW_E_INVALID; }
            if (op->ncws == op->cap_cws) {
                int64_t nc = op->cap_cws ? op->cap_cws * 2 : 1024;
                cw_t* nw = (cw_t*)realloc(op->cws, sizeof(cw_t) * (size_t)nc);
                if (!nw) return GW_E_OOM;
                op->cws = nw;
                op->cap_cws = nc;
            }
            cw_t* w = &op->cws[op->ncws++];
            memset(w, 0, sizeof(*w));
            w->acc0 = (acc_t*)malloc(sizeof(acc_t));
            if (!w->acc0) return GW_E_OOM;
            rd_acc(x + 9 + hb, op->c.agg, w->acc0);
            w->trig = w->total = w->rest = cnt;
        }
        p += (int64_t)m * (17 + hb);
        NEED(4);
        if (rd_be32(p) != 0) { op_err(op, "count windows hold no timers"); return GW_E_INVALID; }
        p += 4;
    }
#undef NEED
    if (p != end) { op_err(op, "snapshot blob has trailing bytes"); return GW_E_INVALID; }
    return GW_OK;
}

/* Returns the blob size; writes it when buf holds >= that many bytes. Negative on error. */
int64_t wo_snapshot(wo_op* op, int32_t kg_lo, int32_t kg_hi, uint8_t* buf, int64_t cap) {
    if (op->c.assigner == GW_COUNT_TUMBLING || op->c.assigner == GW_COUNT_SLIDING)
        return count_snapshot(op, kg_lo, kg_hi, buf, cap);
    if (kg_lo < 0 || kg_hi < kg_lo) return GW_E_INVALID;
    const int nk = kg_hi - kg_lo + 1;
    const int hashed = op->khash.n > 0; /* header flags bit 0: entries carry the key hash */
    /* gather (key group, sort key) for state entries, timers and merging sets */
    int64_t ns = 0, nt = 0, nm = 0;
    snap_ent* se = (snap_ent*)malloc(sizeof(snap_ent) * (size_t)(op->state.n + 1));
    snap_ent* te = (snap_ent*)malloc(sizeof(snap_ent) * (size_t)(op->timers.n + 1));
    snap_ent* me = (snap_ent*)malloc(sizeof(snap_ent) * (size_t)(op->nsets + 1));
    if (!se || !te || !me) { free(se); free(te); free(me); return GW_E_OOM; }
    for (int64_t i = 0; i < op->state.cap; i++) {
        const ment_t* m = &op->state.e[i];
        if (m->st != 1) continue;
        int32_t kg = key_group_of(op, m->k[0]);
        if (kg < kg_lo || kg > kg_hi) continue;
        se[ns++] = (snap_ent){kg, m->k[0], m->k[1], m->k[2], 0, m->v};
    }
    for (int64_t i = 0; i < op->timers.cap; i++) {
        const ment_t* m = &op->timers.e[i];
        if (m->st != 1) continue;
        int32_t kg = key_group_of(op, m->k[1]);
        if (kg < kg_lo || kg > kg_hi) continue;
        te[nt++] = (snap_ent){kg, m->k[1], m->k[2], m->k[3], m->k[0], 0}; /* (key, s, e, ts) */
    }
    for (int64_t i = 0; i < op->sets.cap; i++) {
        const ment_t* m = &op->sets.e[i];
        if (m->st != 1 || op->msets[m->v].n == 0) continue;
        int32_t kg = key_group_of(op, m->k[0]);
        if (kg < kg_lo || kg > kg_hi) continue;
        me[nm++] = (snap_ent){kg, m->k[0], 0, 0, 0, m->v};
    }
    qsort(se, (size_t)ns, sizeof(snap_ent), cmp_snap_ent);
    qsort(te, (size_t)nt, sizeof(snap_ent), cmp_snap_ent);
    qsort(me, (size_t)nm, sizeof(snap_ent), cmp_snap_ent);
    const int64_t hdr = 96, offs_at = hdr, pay0 = hdr + (int64_t)(nk + 1) * 8;
    wbuf b = {buf, pay0, cap};
    int64_t* offs = (int64_t*)calloc((size_t)nk + 1, sizeof(int64_t));
    int64_t a = 0, t = 0, q = 0;
    for (int g = 0; g < nk; g++) {
        const int32_t kg = kg_lo + g;
        offs[g] = b.n - pay0;
        int64_t a1 = a, t1 = t, q1 = q;
        while (a1 < ns && se[a1].kg == kg) a1++;
        while (t1 < nt && te[t1].kg == kg) t1++;
        while (q1 < nm && me[q1].kg == kg) q1++;
        wb_be32(&b, (int32_t)(a1 - a));
        for (; a < a1; a++) { /* namespace, key, [key hash,] state */
            wb_be64(&b, se[a].k1); wb_be64(&b, se[a].k2); wb_be64(&b, se[a].k0);
            if (hashed) wb_be32(&b, key_hash_of(op, se[a].k0));
            wb_acc(&b, op->c.agg, &op->accs[se[a].v]);
            /* minBy / maxBy: the reduced element is the state (HeapReducingState.java:90-97); the
             * GPU writes its payload here (flags bit 1), the oracle its arrival number */
            if (op->c.flags & GW_FLAG_BY_FIELD) wb_be64(&b, op->accs[se[a].v].q);
        }
        wb_be32(&b, (int32_t)(q1 - q));
        for (; q < q1; q++) {
            const mws_t* w = &op->msets[me[q].v];
            /* the list in (window start, end) order: the reference's list order is the
             * mapping's iteration order, which carries no meaning */
            int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * 4 * (size_t)w->n);
            memcpy(idx, w->w, sizeof(int64_t) * 4 * (size_t)w->n);
            for (int i = 1; i < w->n; i++)
                for (int j = i; j > 0 && (idx[4 * j] < idx[4 * j - 4] ||
                                          (idx[4 * j] == idx[4 * j - 4] && idx[4 * j + 1] < idx[4 * j - 3])); j--)
                    for (int c = 0; c < 4; c++) { int64_t x = idx[4 * j + c]; idx[4 * j + c] = idx[4 * j - 4 + c]; idx[4 * j - 4 + c] = x; }
            wb_be64(&b, me[q].k0);
            /* a key whose sessions all fired and purged holds no state entry: the set carries
             * its hash too, so a restore can file it under its key group */
            if (hashed) wb_be32(&b, key_hash_of(op, me[q].k0));
            wb_be32(&b, w->n);
            for (int i = 0; i < 4 * w->n; i++) wb_be64(&b, idx[i]);
            free(idx);
        }
        wb_be32(&b, (int32_t)(t1 - t));
        for (; t < t1; t++) { /* TimerSerializer: flipSignBit(ts), key, namespace */
            wb_be64(&b, (int64_t)((uint64_t)te[t].k3 ^ 0x8000000000000000ull));
            wb_be64(&b, te[t].k0); wb_be64(&b, te[t].k1); wb_be64(&b, te[t].k2);
        }
    }
    offs[nk] = b.n - pay0;
    const int64_t total = b.n;
    if (buf && cap >= total) {
        snap_header(op, kg_lo, kg_hi, hashed, offs[nk], buf);
        memcpy(buf + offs_at, offs, (size_t)(nk + 1) * 8);
    }
    free(offs); free(se); free(te); free(me);
    return total;
}

/* Restore one blob (of any key-group range) into the operator: state entries, merging
 * window sets and timers as the reference's restore reads them back; the watermark stays
 * where it is (Long.MIN_VALUE for a fresh operator). */
int wo_restore(wo_op* op, const uint8_t* buf, int64_t len) {
    if (len < 96 || memcmp(buf, "GWS1", 4) != 0) { op_err(op, "not a snapshot blob"); return GW_E_INVALID; }
    uint32_t ver; int32_t i32s[2], i32b[4]; int64_t i64s[5], tail[3];
    memcpy(&ver, buf + 4, 4); memcpy(i32s, buf + 8, 8); memcpy(i64s, buf + 16, 40);
    memcpy(i32b, buf + 56, 16); memcpy(tail, buf + 72, 24);
    const int64_t slide = op->c.assigner == GW_TUMBLING ? op->c.size : op->c.slide;
    const int32_t mp = op->c.max_parallelism > 0 ? op->c.max_parallelism : 128;
    if (ver != 4 || i32s[0] != op->c.agg || i32s[1] != op->c.assigner || i64s[0] != op->c.size ||
        i64s[1] != slide || i64s[2] != op->c.offset || i64s[3] != op->c.gap || i32b[0] != mp) {
        op_err(op, "snapshot of a different window / aggregate / max parallelism");
        return GW_E_INVALID;
    }
    const int nk = i32b[2] - i32b[1] + 1;
    const int64_t pay0 = 96 + (int64_t)(nk + 1) * 8;
    if (nk <= 0 || tail[2] < 0 || len < pay0 || tail[2] > len - pay0) { op_err(op, "truncated snapshot blob"); return GW_E_INVALID; }
    const uint8_t* p = buf + pay0;
    const uint8_t* end = p + tail[2];
    const int ab = wo_acc_bytes(op->c.agg);
    const int hb = (i64s[4] & 1) ? 4 : 0;
    const int qb = (i64s[4] & 2) ? 8 : 0; /* minBy / maxBy: the element's arrival number */
    if (op->c.assigner == GW_COUNT_TUMBLING) return count_restore(op, p, end, nk, hb);
    if (op->c.assigner == GW_COUNT_SLIDING) { op_err(op, "sliding count windows keep no heap-layout snapshot"); return GW_E_UNSUPPORTED; }
    if (!qb != !(op->c.flags & GW_FLAG_BY_FIELD)) { op_err(op, "minBy / maxBy snapshot into another operator"); return GW_E_INVALID; }
#define NEED(x) do { if ((int64_t)(x) > end - p) { op_err(op, "truncated snapshot blob"); return GW_E_INVALID; } } while (0)
    for (int g = 0; g < nk; g++) {
        NEED(4);
        int32_t n = rd_be32(p); p += 4;
        for (int32_t i = 0; i < n; i++) {
            NEED(24 + hb + ab + qb);
            int64_t s = rd_be64(p), e = rd_be64(p + 8), key = rd_be64(p + 16);
            if (hb) {
                const int32_t kh = rd_be32(p + 24);
                const int rc = wo_set_key_hashes(op, 1, &key, &kh);
                if (rc) return rc;
            }
            acc_t a;
            rd_acc(p + 24 + hb, op->c.agg, &a);
            a.q = qb ? rd_be64(p + 24 + hb + ab) : 0;
            p += 24 + hb + ab + qb;
            int64_t k[4] = {key, s, e, 0};
            int created = 0;
            ment_t* m = map_upsert(&op->state, k, -1, &created);
            if (!m) return GW_E_OOM;
            if (created) {
                int64_t ai = acc_alloc(op);
                if (ai < 0) return GW_E_OOM;
                m = map_find(&op->state, k);
                m->v = ai;
                op->accs[ai] = a;
            } else {
                acc_merge(&op->accs[m->v], &a, op->c.agg);
            }
        }
        NEED(4);
        int32_t nm = rd_be32(p); p += 4;
        for (int32_t i = 0; i < nm; i++) {
            NEED(12 + hb);
            int64_t key = rd_be64(p);
            if (hb) {
                const int32_t kh = rd_be32(p + 8);
                const int rc = wo_set_key_hashes(op, 1, &key, &kh);
                if (rc) return rc;
            }
            int32_t c = rd_be32(p + 8 + hb);
            p += 12 + hb;
            NEED((int64_t)c * 32);
            mws_t* w = mws_get(op, key, 1);
            for (int32_t j = 0; j < c; j++, p += 32)
                mws_put(w, rd_be64(p), rd_be64(p + 8), rd_be64(p + 16), rd_be64(p + 24));
        }
        NEED(4);
        int32_t t = rd_be32(p); p += 4;
        for (int32_t i = 0; i < t; i++, p += 32) {
            NEED(32);
            int64_t ts = (int64_t)((uint64_t)rd_be64(p) ^ 0x8000000000000000ull);
            int rc = tmr_register(op, rd_be64(p + 8), rd_be64(p + 16), rd_be64(p + 24), ts);
            if (rc) return rc;
        }
    }
#undef NEED
    return GW_OK;
}

/* ------------------------------------------------------------------------ */
/* multi-threaded CPU baseline: one operator per simulated subtask            */
/* ------------------------------------------------------------------------ */
typedef struct {
    const gw_config* cfg;
    int idx, threads;
    int64_t nb;
    const int64_t *blen, *wm, *key, *ts, *val;
    int64_t rows, checksum;
    int64_t* pw_rows;  /* optional [nb + 1]: rows fired per watermark (the last: MAX_WATERMARK) */
    uint64_t* pw_cs;   /* optional [nb + 1]: order-independent checksum of those rows */
    int rc;
    int no_final;      /* 1: no MAX_WATERMARK after the last batch (the stream's own cadence) */
    int keep_rows;     /* 1: keep every row (rk.. / rwm, nrows of rcap) */
    int64_t *rk, *rs, *re, *rr;
    int32_t* rwm;
    int64_t nrows, rcap;
} par_arg;

static int keep_row_buf(par_arg* a, int64_t more) {
    if (a->nrows + more <= a->rcap) return 0;
    int64_t cap = a->rcap ? a->rcap : 1 << 16;
    while (cap < a->nrows + more) cap *= 2;
    int64_t* b[4] = {a->rk, a->rs, a->re, a->rr};
    for (int c = 0; c < 4; c++) {
        int64_t* nb = (int64_t*)realloc(b[c], (size_t)cap * 8);
        if (!nb) return GW_E_OOM;
        b[c] = nb;
    }
    a->rk = b[0]; a->rs = b[1]; a->re = b[2]; a->rr = b[3];
    int32_t* w = (int32_t*)realloc(a->rwm, (size_t)cap * 4);
    if (!w) return GW_E_OOM;
    a->rwm = w;
    a->rcap = cap;
    return 0;
}

static void* par_main(void* p) {
    par_arg* a = (par_arg*)p;
    wo_op* op = wo_create(a->cfg);
    if (!op) { a->rc = GW_E_OOM; return NULL; }
    int32_t maxp = a->cfg->max_parallelism > 0 ? a->cfg->max_parallelism : 128;
    int64_t off = 0, rows = 0;
    uint64_t cs = 0;
    int64_t* bk = (int64_t*)malloc(4 * 8 * 1024);
    int64_t* bs = bk + 1024;
    int64_t* be = bs + 1024;
    int64_t* br = be + 1024;
    for (int64_t b = 0; b <= a->nb; b++) {
        if (b == a->nb && a->no_final) break;
        if (b < a->nb) {
            for (int64_t i = off; i < off + a->blen[b]; i++) {
                int32_t kg = wo_assign_to_key_group(wo_long_hash(a->key[i]), maxp);
                if (wo_operator_index_for_key_group(maxp, a->threads, kg) != a->idx) continue;
                int rc = wo_process_element(op, a->key[i], a->ts[i], a->val ? a->val[i] : 0);
                if (rc) { a->rc = rc; goto done; }
            }
            off += a->blen[b];
        }
        int rc = wo_process_watermark(op, b < a->nb ? a->wm[b] : INT64_MAX);
        if (rc) { a->rc = rc; goto done; }
        int64_t n;
        while ((n = wo_drain(op, bk, bs, be, br, 1024)) > 0) {
            uint64_t c = 0;
            for (int64_t i = 0; i < n; i++)
                c += (uint64_t)bk[i] * 0x9e3779b97f4a7c15ull ^ (uint64_t)bs[i] * 31u ^
                     (uint64_t)be[i] * 17u ^ (uint64_t)br[i];
            cs += c;
            rows += n;
            if (a->pw_rows) { a->pw_rows[b] += n; a->pw_cs[b] += c; }
            if (a->keep_rows) {
                if (keep_row_buf(a, n)) { a->rc = GW_E_OOM; goto done; }
                memcpy(a->rk + a->nrows, bk, (size_t)n * 8);
                memcpy(a->rs + a->nrows, bs, (size_t)n * 8);
                memcpy(a->re + a->nrows, be, (size_t)n * 8);
                memcpy(a->rr + a->nrows, br, (size_t)n * 8);
                for (int64_t i = 0; i < n; i++) a->rwm[a->nrows + i] = (int32_t)b;
                a->nrows += n;
            }
        }
    }
done:
    free(bk);
    a->rows = rows;
    a->checksum = (int64_t)cs;
    wo_destroy(op);
    return NULL;
}

static int64_t run_parallel(const gw_config* cfg, int threads, int64_t nb, const int64_t* blen,
                            const int64_t* wm, const int64_t* key, const int64_t* ts,
                            const int64_t* val, int no_final, int64_t* checksum, double* seconds) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    par_arg* args = (par_arg*)calloc((size_t)threads, sizeof(par_arg));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; i++) {
        args[i] = (par_arg){cfg, i, threads, nb, blen, wm, key, ts, val, 0, 0, NULL, NULL, 0, no_final, 0, NULL, NULL, NULL, NULL, NULL, 0, 0};
        pthread_create(&th[i], NULL, par_main, &args[i]);
    }
    int64_t rows = 0;
    uint64_t cs = 0;
    int rc = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        rows += args[i].rows;
        cs += (uint64_t)args[i].checksum;
        if (args[i].rc) rc = args[i].rc;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (checksum) *checksum = (int64_t)cs;
    free(th);
    free(args);
    return rc ? rc : rows;
}

int64_t wo_run_parallel(const gw_config* cfg, int threads, int64_t nb, const int64_t* blen,
                        const int64_t* wm, const int64_t* key, const int64_t* ts,
                        const int64_t* val, int64_t* checksum, double* seconds) {
    return run_parallel(cfg, threads, nb, blen, wm, key, ts, val, 0, checksum, seconds);
}

/* The same without the final MAX_WATERMARK: the batches at the stream's own watermark cadence
 * only (what a bench's timed steps do). */
int64_t wo_run_parallel_stream(const gw_config* cfg, int threads, int64_t nb, const int64_t* blen,
                               const int64_t* wm, const int64_t* key, const int64_t* ts,
                               const int64_t* val, int64_t* checksum, double* seconds) {
    return run_parallel(cfg, threads, nb, blen, wm, key, ts, val, 1, checksum, seconds);
}

/* wo_run_parallel with per-watermark results: wm_rows[b] / wm_cs[b] (b = 0..nb, the last
 * entry for the final MAX_WATERMARK) receive the number of rows each watermark fired over
 * all subtasks and the sum of their row hashes (the checksum of wo_run_parallel, per
 * watermark) -- what a GPU run's per-watermark output is compared against at full size. */
int64_t wo_run_parallel_wm(const gw_config* cfg, int threads, int64_t nb, const int64_t* blen,
                           const int64_t* wm, const int64_t* key, const int64_t* ts, const int64_t* val,
                           int64_t* wm_rows, int64_t* wm_cs, double* seconds) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    par_arg* args = (par_arg*)calloc((size_t)threads, sizeof(par_arg));
    int64_t* pr = (int64_t*)calloc((size_t)threads * (size_t)(nb + 1), sizeof(int64_t));
    uint64_t* pc = (uint64_t*)calloc((size_t)threads * (size_t)(nb + 1), sizeof(uint64_t));
    if (!th || !args || !pr || !pc) { free(th); free(args); free(pr); free(pc); return GW_E_OOM; }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; i++) {
        args[i] = (par_arg){cfg, i, threads, nb, blen, wm, key, ts, val, 0, 0,
                            pr + (size_t)i * (size_t)(nb + 1), pc + (size_t)i * (size_t)(nb + 1), 0, 0, 0, NULL, NULL, NULL, NULL, NULL, 0, 0};
        pthread_create(&th[i], NULL, par_main, &args[i]);
    }
    int64_t rows = 0;
    int rc = 0;
    for (int64_t b = 0; b <= nb; b++) { wm_rows[b] = 0; wm_cs[b] = 0; }
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        rows += args[i].rows;
        if (args[i].rc) rc = args[i].rc;
        for (int64_t b = 0; b <= nb; b++) {
            wm_rows[b] += args[i].pw_rows[b];
            wm_cs[b] = (int64_t)((uint64_t)wm_cs[b] + args[i].pw_cs[b]);
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    free(th); free(args); free(pr); free(pc);
    return rc ? rc : rows;
}

/* wo_run_parallel keeping every fired row: (key, start, end, result bits, watermark index)
 * into the caller's arrays of cap rows (the last watermark index nb = MAX_WATERMARK).
 * Returns the number of rows, GW_E_OUTPUT_FULL (nothing written) if more than cap. */
int64_t wo_run_parallel_rows(const gw_config* cfg, int threads, int64_t nb, const int64_t* blen,
                             const int64_t* wm, const int64_t* key, const int64_t* ts, const int64_t* val,
                             int64_t cap, int64_t* ok, int64_t* os, int64_t* oe, int64_t* orr, int32_t* owm,
                             double* seconds) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    par_arg* args = (par_arg*)calloc((size_t)threads, sizeof(par_arg));
    if (!th || !args) { free(th); free(args); return GW_E_OOM; }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; i++) {
        memset(&args[i], 0, sizeof(par_arg));
        args[i].cfg = cfg; args[i].idx = i; args[i].threads = threads; args[i].nb = nb; args[i].blen = blen;
        args[i].wm = wm; args[i].key = key; args[i].ts = ts; args[i].val = val; args[i].keep_rows = 1;
        pthread_create(&th[i], NULL, par_main, &args[i]);
    }
    int64_t total = 0;
    int rc = 0;
    for (int i = 0; i < threads; i++) {
        pthread_join(th[i], NULL);
        total += args[i].nrows;
        if (args[i].rc) rc = args[i].rc;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds) *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (!rc && total > cap) rc = GW_E_OUTPUT_FULL;
    int64_t at = 0;
    for (int i = 0; i < threads; i++) {
        par_arg* a = &args[i];
        if (!rc && a->nrows) {
            memcpy(ok + at, a->rk, (size_t)a->nrows * 8);
            memcpy(os + at, a->rs, (size_t)a->nrows * 8);
            memcpy(oe + at, a->re, (size_t)a->nrows * 8);
            memcpy(orr + at, a->rr, (size_t)a->nrows * 8);
            memcpy(owm + at, a->rwm, (size_t)a->nrows * 4);
            at += a->nrows;
        }
        free(a->rk); free(a->rs); free(a->re); free(a->rr); free(a->rwm);
    }
    free(th); free(args);
    return rc ? rc : total;
}

/* ---------------------------------------------------------------------------
 * Network-buffer decode, one input channel, sequential —
 * the way the reference's record deserializer walks a buffer:
 *   - length word: NonSpanningWrapper.readInt = getIntBigEndian
 *     (flink-runtime/.../io/network/api/serialization/NonSpanningWrapper.java:142-144);
 *     a record that does not fit the remaining bytes waits for the next buffer
 *     (hasCompleteLength / canReadRecord :351-357, SpanningWrapper);
 *   - element: StreamElementSerializer.deserialize
 *     (RS/runtime/streamrecord/StreamElementSerializer.java:200-225): tag byte, then
 *     REC_WITH_TIMESTAMP (0): long ts + value; REC_WITHOUT_TIMESTAMP (1): value;
 *     WATERMARK (2): long; INTERNAL_WATERMARK (6): int subpartition + long;
 *     STREAM_STATUS (4): int; LATENCY_MARKER (3): long, long, long, int;
 *     RECORD_ATTRIBUTES (5): boolean; any other tag: "Corrupt stream" IOException;
 *   - value: TupleSerializer.serialize writes the fields in order
 *     (flink-core/.../api/java/typeutils/runtime/TupleSerializer.java:135-144), each
 *     with its DataOutputView primitive (big-endian).
 * A record without timestamp carries Long.MIN_VALUE (StreamRecord.getTimestamp).
 * ------------------------------------------------------------------------- */
static int field_width(char t) {
    switch (t) {
        case 'J': case 'D': return 8;
        case 'I': case 'F': return 4;
        case 'S': return 2;
        case 'B': case 'Z': return 1;
        default: return -1;
    }
}

static uint64_t be_read(const uint8_t* p, int w) {
    uint64_t v = 0;
    for (int i = 0; i < w; i++) v = (v << 8) | p[i];
    return v;
}

/* field -> the 8-byte value column: integral types sign-extended to int64,
 * float widened to double (Java's float -> double conversion is exact). */
static int64_t field_to_bits(char t, const uint8_t* p) {
    uint64_t u = be_read(p, field_width(t));
    switch (t) {
        case 'J': case 'D': return (int64_t)u;
        case 'I': return (int64_t)(int32_t)(uint32_t)u;
        case 'S': return (int64_t)(int16_t)(uint16_t)u;
        case 'B': return (int64_t)(int8_t)(uint8_t)u;
        case 'Z': return (int64_t)(u != 0);
        case 'F': {
            uint32_t b = (uint32_t)u;
            float f;
            double d;
            int64_t r;
            memcpy(&f, &b, 4);
            d = (double)f;
            memcpy(&r, &d, 8);
            return r;
        }
    }
    return 0;
}

int wo_decode_stream(const uint8_t* buf, int64_t nbytes, const gw_record_layout* lay,
                     int64_t* key, int64_t* ts, int64_t* value_bits, int64_t rec_cap,
                     int64_t* wm_pos, int64_t* wm_val, int64_t wm_cap, gw_decode_result* out) {
    if (!lay || lay->nfields < 1 || lay->nfields > GW_MAX_FIELDS) return GW_E_INVALID;
    int off[GW_MAX_FIELDS], vbytes = 0;
    for (int i = 0; i < lay->nfields; i++) {
        int w = field_width(lay->types[i]);
        if (w < 0) return GW_E_INVALID;
        off[i] = vbytes;
        vbytes += w;
    }
    if (lay->key_field < 0 || lay->key_field >= lay->nfields || lay->types[lay->key_field] != 'J')
        return GW_E_INVALID;
    if (lay->value_field >= lay->nfields) return GW_E_INVALID;
    int64_t pos = 0, nr = 0, nw = 0, sk = 0;
    while (pos + 4 <= nbytes) {
        int64_t len = (int32_t)(uint32_t)be_read(buf + pos, 4);
        if (len < 1) return GW_E_INVALID;
        if (len + 4 > GW_MAX_ELEMENT) return GW_E_UNSUPPORTED; /* valid in Flink, beyond the GPU decoder */
        if (pos + 4 + len > nbytes) break; /* spans into the next buffer */
        const uint8_t* e = buf + pos + 4;
        int tag = e[0];
        if (tag == 0 || tag == 1) {
            int hdr = tag == 0 ? 9 : 1;
            if (len != hdr + vbytes) return GW_E_INVALID;
            if (nr >= rec_cap) return GW_E_OUTPUT_FULL;
            const uint8_t* v = e + hdr;
            ts[nr] = tag == 0 ? (int64_t)be_read(e + 1, 8) : INT64_MIN;
            key[nr] = (int64_t)be_read(v + off[lay->key_field], 8);
            if (value_bits)
                value_bits[nr] = lay->value_field >= 0
                                     ? field_to_bits(lay->types[lay->value_field], v + off[lay->value_field])
                                     : 0;
            nr++;
        } else if (tag == 2 || tag == 6) {
            if (len != (tag == 2 ? 9 : 13)) return GW_E_INVALID;
            if (nw >= wm_cap) return GW_E_OUTPUT_FULL;
            wm_pos[nw] = nr;
            wm_val[nw] = (int64_t)be_read(e + (tag == 2 ? 1 : 5), 8);
            nw++;
        } else if (tag == 3 || tag == 4 || tag == 5) {
            if (len != (tag == 3 ? 29 : tag == 4 ? 5 : 2)) return GW_E_INVALID;
            sk++;
        } else {
            return GW_E_INVALID;
        }
        pos += 4 + len;
    }
    if (out) {
        out->records = nr;
        out->watermarks = nw;
        out->consumed = pos;
        out->skipped = sk;
    }
    return GW_OK;
}
