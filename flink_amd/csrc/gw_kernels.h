// gw_kernels.h — pane-table layout, kernel argument blocks and launcher declarations.
//
// Pane state table: `cap` slots in `nreg` regions of S = 2^log2S slots,
// plus one sentinel region (slot index `cap`) for the key Long.MIN_VALUE, which doubles
// as the empty marker.  The regions form 2^rb1 buckets of `nsub` regions each (nsub need not
// be a power of two, so the table can sit at load ~0.8 instead of a power of two at <= 0.7):
// a key's bucket is the top rb1 bits of its hash, its region within the bucket the next 32
// bits scaled to nsub (multiply-high), its home slot the low bits; linear probing stays
// inside the region.  Each region is stored SoA:
//
//     keys [S]                int64, kEmptyKey while free (set once by CAS)
//     mask [S]                presence bits per ring cell (SUM/MIN/MAX only), 1/2/4/8
//                             bytes per slot as the ring length R needs (Q5: R = 6, 1 B)
//     cells[R][S][W]          pane accumulators, pane-major (W = 2 for AVG)
//
// so an ingest pass touches only the keys, the mask and the 1-2 pane arrays the batch
// hits, each as one contiguous block per region (loaded into LDS and written back whole
// by k_rgn_apply), and a fire pass streams every array coalesced.
#pragma once
#include "gw_device.h"

namespace gw {

struct PaneTable {
    int64_t* base;
    int64_t cap;           // slots = nreg << log2S (sentinel slot index = cap)
    int64_t nreg;          // regions = nsub << rb1, + 1 sentinel region allocated
    int64_t region_words;  // S + mask words + S * R * W
    int32_t log2S;
    int32_t rb1;           // bucket bits: the pass-1 buckets of the region path (0: one region)
    int32_t nsub;          // regions per bucket (1: single-pass table)
    int32_t ring;          // R
    int32_t words;         // W
    int32_t agg;
    int32_t has_mask;
    int32_t mask_shift;    // log2 bytes of one slot's presence mask
};

GW_HD int64_t pt_S(const PaneTable& t) { return (int64_t)1 << t.log2S; }
GW_HD int64_t* pt_region(const PaneTable& t, int64_t r) { return t.base + r * t.region_words; }
GW_HD int64_t* pt_key(const PaneTable& t, int64_t g) {
    return pt_region(t, g >> t.log2S) + (g & (pt_S(t) - 1));
}
// int64 words of one region's mask array (S >= 16, so always a whole, even number)
GW_HD int64_t pt_mask_words(const PaneTable& t) { return t.has_mask ? (pt_S(t) << t.mask_shift) >> 3 : 0; }
GW_HD uint8_t* pt_mask_base(const PaneTable& t, int64_t r) { return (uint8_t*)(pt_region(t, r) + pt_S(t)); }
GW_HD int64_t* pt_cell(const PaneTable& t, int64_t g, int pos) {
    const int64_t S = pt_S(t);
    return pt_region(t, g >> t.log2S) + S + pt_mask_words(t) + ((int64_t)pos * S + (g & (S - 1))) * t.words;
}
// Presence mask of slot j in a region's mask array m (global or LDS).
__device__ __forceinline__ uint64_t mask_get(const uint8_t* m, int64_t j, int shift) {
    switch (shift) {
    case 0: return m[j];
    case 1: return ((const uint16_t*)m)[j];
    case 2: return ((const uint32_t*)m)[j];
    default: return ((const uint64_t*)m)[j];
    }
}
__device__ __forceinline__ void mask_put(uint8_t* m, int64_t j, int shift, uint64_t v) {
    switch (shift) {
    case 0: m[j] = (uint8_t)v; break;
    case 1: ((uint16_t*)m)[j] = (uint16_t)v; break;
    case 2: ((uint32_t*)m)[j] = (uint32_t)v; break;
    default: ((uint64_t*)m)[j] = v; break;
    }
}
// Atomically set presence bit `pos` of slot j (32-bit atomic on the word holding it);
// returns true if the bit was clear.
__device__ __forceinline__ bool mask_set_bit(uint8_t* m, int64_t j, int shift, uint32_t pos) {
    const uint64_t bit = ((uint64_t)j << (shift + 3)) + pos;
    uint32_t* w = (uint32_t*)m + (bit >> 5);
    const uint32_t b = 1u << (bit & 31);
    if (*w & b) return false;  // bits only get set: a stale read is a clear bit, which the OR resolves
    return !(atomicOr(w, b) & b);
}
__device__ __forceinline__ uint64_t pt_mask_get(const PaneTable& t, int64_t g) {
    return mask_get(pt_mask_base(t, g >> t.log2S), g & (pt_S(t) - 1), t.mask_shift);
}
__device__ __forceinline__ void pt_mask_put(const PaneTable& t, int64_t g, uint64_t v) {
    mask_put(pt_mask_base(t, g >> t.log2S), g & (pt_S(t) - 1), t.mask_shift, v);
}
// bucket, region within the bucket, region and home slot of a key hash (independent bit
// ranges: the top rb1 bits, the 32 below them, the low log2S)
GW_HD int64_t pt_bucket(const PaneTable& t, uint64_t h) { return t.rb1 == 0 ? 0 : (int64_t)(h >> (64 - t.rb1)); }
// also valid on a compact region word (its top rb1 bits replaced, gw_pane.hip cmp_pack)
GW_HD int32_t pt_sub(const PaneTable& t, uint64_t h) {
    const uint32_t u = (uint32_t)((h << t.rb1) >> 32);
    return (int32_t)(((uint64_t)u * (uint32_t)t.nsub) >> 32);
}
GW_HD int64_t pt_key_region(const PaneTable& t, uint64_t h) {
    return t.nsub == 1 ? pt_bucket(t, h) : pt_bucket(t, h) * t.nsub + pt_sub(t, h);
}
// The home slot is aligned to a group of kProbeGroup slots: linear probing then starts
// on a 32-B group boundary, so k_rgn_apply compares a whole group of keys per LDS step
// (one probe step for almost every key at the table's load) with the same slot order
// as the scalar probes of the other kernels.
constexpr int kProbeGroup = 4;
GW_HD int64_t pt_home(const PaneTable& t, uint64_t h) {
    return (int64_t)(h & (uint64_t)(pt_S(t) - 1) & ~(uint64_t)(kProbeGroup - 1));
}

// Find (or insert) the slot of `key` in its region; -1 if the probe limit is hit.
__device__ __forceinline__ int64_t pt_find_or_insert(const PaneTable& t, int64_t key, bool& inserted) {
    inserted = false;
    if (key == kEmptyKey) return t.cap;
    const uint64_t h = slot_hash(key);
    const int64_t S = pt_S(t);
    const int64_t r = pt_key_region(t, h);
    int64_t* keys = pt_region(t, r);
    int64_t j = pt_home(t, h);
    const int lim = S < kMaxProbe ? (int)S : kMaxProbe;
    for (int p = 0; p < lim; ++p) {
        int64_t* kp = keys + j;
        const int64_t k = *kp;  // stale only as kEmptyKey (find_or_insert)
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

struct IngestArgs {
    const int64_t* key;
    const int64_t* ts;
    const int64_t* val;
    int64_t n;
    // packed exchange words (gw_ingest_packed_device): records [pk_from, n) are pk_w[i -
    // pk_from], decoded by the region P1 itself (unpack_word: key, pane start, value)
    const uint64_t* pk_w;
    int64_t pk_from;
    gw_pack_geom pk_g;
    int64_t t_late;     // first non-late timestamp (start of the first unfired window)
    int64_t p_late;     // its pane index
    uint64_t delta;     // ring base pane B - p_late (>= 0)
    uint64_t q_refire;  // lateness > 0: panes p_late .. p_late + q_refire - 1 belong to fired,
                        // not yet cleaned windows; their records go to the re-fire list
    int64_t seq0;       // arrival number of record 0 of this call (re-fire order)
    int64_t* lo_key;    // late side output (WindowOperator.sideOutput :587-588), append at
    int64_t* lo_ts;     //   st->n_late_out; nullptr: late records are counted and dropped
    int64_t* lo_val;
    int64_t* rf_key;    // re-fire list (append at st->n_refire)
    int64_t* rf_pane;
    int64_t* rf_a0;
    int64_t* rf_a1;
    int64_t* rf_seq;
    UDiv64 div;         // division by the pane width g
    int32_t b_pos;      // B mod R
    int32_t late_exact; // 0: t_late was clamped at Long.MIN_VALUE (then ts < t_late is a range error)
    PaneTable t;
    // window class of a composite handle (gw_runtime.cpp, rings beyond kMaxRing): this
    // operator holds the windows k = j (mod J) of slide `cls_slide`, offset `cls_off`; a late
    // record is counted / side-output only by the class of its last window
    int64_t cls_slide;
    int64_t cls_off;
    int32_t cls_J;      // 0 or 1: not a window class
    int32_t cls_j;
    // size < slide (gw_runtime.cpp: pane width = slide, one pane per window): a record whose
    // offset in its pane is >= gap_size lies between two windows and belongs to none
    int64_t gap_w;      // pane width (= slide) when gap_size > 0
    int64_t gap_size;   // window size, 0: no gaps
    int64_t gap_late;   // a record in a gap is late iff ts <= gap_late (= watermark - lateness:
                        // isElementLate, WindowOperator.java:620-623)
    int64_t* d_key;     // deferred list (append at st->n_deferred)
    int64_t* d_pane;
    int64_t* d_a0;
    int64_t* d_a1;
    DevStatus* st;
    // region path (k_rgn_p1 / k_rgn_plan* / k_rgn_p2 / k_rgn_apply, gw_pane.hip)
    int32_t d1_bits;       // region = pass-1 bucket * nsub + pass-2 bucket (t.rb1, t.nsub)
    int32_t two_pass;      // 0: single-pass table, nsub = 1 (apply reads the P1 tiles directly)
    int32_t fmt;           // region record format (gw_pane.hip): 0 wide, 1 compact (hash word +
                           // 32-bit value), 2 narrow (32-bit key + 28-bit value; 4 B for COUNT)
    int32_t nar2;          // narrow two-pass flushes (k_rgn_apply_nar): P2 groups each round by
                           // (super-region, ring position); one workgroup per super-region of
    int32_t sr_bits;       //   2^sr_bits probe regions applies one ring position after another
    // nar2 carry (gw_runtime.cpp flush_buffer): a fire's flush applies only the ring positions
    // the fire needs (apply_mask); the others stay in its P2 output and the next flush applies
    // them from there (c_*: that output, c_mask: its carried positions)
    uint64_t apply_mask;
    uint64_t c_mask;
    const int64_t* c_rbeg;
    const uint32_t* c_r_row;
    const int64_t* c_r_base;
    int64_t* c_key;
    int32_t cur_empty;     // no current segments: the carried positions alone
    int64_t tile0;         // P1: buffer tile of this batch's first tile
    int64_t ntiles;        // flush: buffer tiles in use
    int64_t ngroups;       // flush: P1 tile groups (= P2 blocks per bucket)
    int32_t p2_group;      // flush: P1 tiles per group (G)
    int64_t* p1_key;       // P1 output: tile t at [t * kPartTile, ...), sorted by bucket
    int64_t* p1_a0;
    int64_t* p1_a1;
    uint8_t* p1_pos;
    uint32_t* p1_row;      // [tile][kPartBuckets] (start << 16 | count) per bucket
    uint32_t* p2_desc;     // [bucket][tile]  the same descriptors, transposed
    int64_t* p2_off;       // [bucket * ngroups + group] sizes -> output starts within the bucket
    int64_t* p2_roff;      // [bucket * ngroups + group] rounds -> first round within the bucket
    int64_t* rbeg;         // [nb1 + 1] first P2 round of each bucket
    int64_t* bk_off;       // [nb1 + 1] first P2 output record of each bucket
    int64_t* e_key;        // P2 output, bucket-major, rounds sorted by region
    int64_t* e_a0;
    int64_t* e_a1;
    uint8_t* e_pos;
    uint32_t* r_row;       // [round][kPartBuckets] (start << 16 | count) per region of the bucket
    int64_t* r_base;       // [round] first record of the round
    unsigned long long* batch_occ;  // ring positions the buffered records touch (for k_rgn_apply)
    DevStatus* st_host;             // buffered P1: pinned host slot k_publish_status copies the status into
    unsigned long long st_seq;      //     and the stamp it writes last
    uint64_t ring_fresh;            // ring positions holding only identities (not in occ)
    int32_t stale;                  // lazily retired cells may hold stale values behind clear presence bits
};

#ifndef GW_PART_TILE
#define GW_PART_TILE 4096
#endif
constexpr int kPartTile = GW_PART_TILE;  // records per P1 tile / P2 round (LDS-sorted)
constexpr int kPartBuckets = 256;   // descriptor row width (<= 8 region bits per pass)
constexpr int kRgnMaxRegions = 65536;
constexpr int kMaxGroup = 256;      // P1 tiles per P2 block (G = 7/4 of the pass-1 buckets; LDS keeps 4 blocks per CU)

struct MergeArgs {
    const int64_t* i_key;
    const int64_t* i_pane;
    const int64_t* i_a0;
    const int64_t* i_a1;
    int64_t n;
    int64_t b;          // ring base pane
    int32_t b_pos;
    PaneTable t;
    int64_t* d_key;     // entries still outside the ring (append at st->n_deferred)
    int64_t* d_pane;
    int64_t* d_a0;
    int64_t* d_a1;
    DevStatus* st;
};

// Restored window state (allowed by a heap-layout snapshot, gw_restore): one entry per
// restored (key, window) state entry of the reference, sorted by (key, window index), each
// key's entries reachable from its slot through head[slot] (-1: none).  A restored window
// fires as the fold of its accumulator and the panes of the records that arrived after the
// restore.
constexpr uint32_t kOvTimer = 1;  // its event-time timer (maxTimestamp) is pending
constexpr uint32_t kOvDead = 2;   // its state was purged
struct Overlay {
    const int32_t* head;  // [cap + 1], nullptr when no restored state is left
    const int64_t* key;
    const int64_t* k;     // window index: start = offset + k * slide
    const int64_t* a0;
    const int64_t* a1;
    uint32_t* flags;
    int64_t n;
    int32_t purge;        // fired windows lose their state (lateness 0 or PurgingTrigger)
};

struct FireArgs {
    PaneTable t;
    Overlay ov;
    int64_t k0;         // window index of the first window of this pass
    int32_t nwin;
    int64_t start0;     // start of the first window fired in this pass
    int64_t slide;
    int64_t size;
    uint64_t rmask;     // ring positions retired after this pass
    int32_t lazy_retire;  // presence-mask aggregates: retiring clears the mask bits only; the
                          // cells keep stale values behind clear bits (gw_runtime.cpp stale_pos)
    int32_t guarded;      // launched behind k_fire_guard: do nothing when st->fire_skip is set
    uint64_t wmask[kMaxRing];
    int64_t* o_key;
    int64_t* o_start;
    int64_t* o_end;
    int64_t* o_res;
    DevStatus* st;
};

// Late records of fired, not yet cleaned windows (allowed lateness > 0), in (key, arrival)
// order: each emits one row per such window it belongs to (EventTimeTrigger.onElement FIRE,
// RS/api/windowing/triggers/EventTimeTrigger.java:37-45; WindowOperator.java:408-446).
struct RefireArgs {
    PaneTable t;
    Overlay ov;
    int64_t n;
    const uint32_t* order;  // entry indices sorted by (key, seq)
    const int64_t* rf_key;
    const int64_t* rf_pane;
    const int64_t* rf_a0;
    const int64_t* rf_a1;
    int64_t b;              // ring base pane
    int32_t b_pos;
    int32_t purging;        // PurgingTrigger: a late record's row holds the record alone
    int64_t m, np;          // slide and size in panes
    int64_t k_lo, k_hi;     // windows that re-fire: k_lo .. k_hi (not late, already fired)
    int64_t offset, slide, size;
    int64_t* o_key;
    int64_t* o_start;
    int64_t* o_end;
    int64_t* o_res;
    DevStatus* st;
};

struct EvictArgs {
    PaneTable t;
    uint64_t emask;
    int64_t pane_of_pos[kMaxRing];
    int64_t* d_key;
    int64_t* d_pane;
    int64_t* d_a0;
    int64_t* d_a1;
    DevStatus* st;
};

struct SnapArgs {
    PaneTable t;
    uint64_t occ;                  // ring positions that may hold data
    int64_t pane_of_pos[kMaxRing]; // pane index held by each ring position
    const int64_t* d_key;          // deferred list
    const int64_t* d_pane;
    const int64_t* d_a0;
    const int64_t* d_a1;
    int64_t n_def;
    int32_t max_p, kg_lo, kg_hi;
    int64_t* o_key;                // collected entries (append at *n_out)
    int64_t* o_pane;
    int64_t* o_a0;
    int64_t* o_a1;
    int32_t* o_kg;
    unsigned long long* n_out;
};
hipError_t launch_snap_collect(const SnapArgs& a, hipStream_t s);

hipError_t launch_table_init(const PaneTable& t, hipStream_t s);
// Insert every overlay key into the table and point head[slot] at its first entry.
hipError_t launch_overlay_attach(const PaneTable& t, const Overlay& ov, int32_t* head, DevStatus* st, hipStream_t s);
// path: 0 direct atomics, 1 LDS pre-aggregation (the region path has its own launchers)
hipError_t launch_ingest(const IngestArgs& a, int path, int unroll, hipStream_t s);
// region path: P1 over one batch (a.n records -> buffer tiles from a.tile0) ...
// e0 / e1 (timing, may be null): events stamped with the first kernel's start and the last
// kernel's end of the launch (hipExtLaunchKernelGGL), so a timed launch measures its kernels
// without the marker packets of hipEventRecord around them.
hipError_t launch_region_p1(const IngestArgs& a, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
hipError_t launch_publish_status(const IngestArgs& a, hipStream_t s);
// ... and, per flush, plan + P2 (two-pass tables) + apply over a.ntiles buffer tiles
hipError_t launch_region_flush(const IngestArgs& a, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
// ... and after a flush that filled regions: its spilled records -> the deferred list
hipError_t launch_region_collect(const IngestArgs& a, hipStream_t s);
int region_group(int d1_bits);  // G: P1 tiles per P2 block
hipError_t launch_merge_deferred(const MergeArgs& a, hipStream_t s);
hipError_t launch_refire(const RefireArgs& a, hipStream_t s);
// re-fire sort keys: mode 0 k[i] = seq[i] - seq_base, v[i] = i; mode 1 k[i] = key[v[i]]
hipError_t launch_refire_keys(int mode, const int64_t* src, int64_t base, uint64_t* k, uint32_t* v, int64_t n,
                              hipStream_t s);
hipError_t launch_deferred_min(const int64_t* pane, int64_t n, DevStatus* st, hipStream_t s);
hipError_t launch_fire(const FireArgs& a, hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
// The checks that let a fire be enqueued right behind a flush, without the host reading the
// status in between (gw_runtime.cpp fast_fire): st->fire_skip = 1 -- the guarded fire does
// nothing and the host takes the exact path -- when the flush left spilled or wide records or
// a full table, when the deferred list does not hold expect_ndef entries, when a record error
// was flagged, or when the fire's rows could exceed the row buffer (the host's own
// ensure_output test, on the device counters); st->fire_rows0 = the output cursor.
struct FireGuard {
    unsigned long long expect_ndef;
    int64_t o_cap;
    int64_t nwin;
    int64_t reset_rows;  // first zero the row cursor (a gw_clear_rows the host deferred to here)
};
hipError_t launch_fire_guard(DevStatus* st, const FireGuard& g, hipStream_t s);
// Cells of ring positions `pmask` whose presence bit is clear -> the identity (the retires a
// lazy fire left behind, before a kernel that adds into cells with device atomics)
hipError_t launch_clean_stale(const PaneTable& t, uint64_t pmask, hipStream_t s);
hipError_t launch_evict(const EvictArgs& a, hipStream_t s);
hipError_t launch_rehash(const PaneTable& o, const PaneTable& n, DevStatus* st, hipStream_t s);
hipError_t launch_status_set(DevStatus* st, int word, unsigned long long v, int shard_field, hipStream_t s);
hipError_t launch_count_live(const PaneTable& t, unsigned long long* out, hipStream_t s);

// key groups / exchange (gw_keygroups.hip)
hipError_t launch_key_groups(int64_t n, const int64_t* key, const int32_t* key_hash, int32_t max_p,
                             int32_t p, int32_t* kg, int32_t* owner, hipStream_t s);
int64_t partition_scratch_bytes(int64_t n, int32_t p);
// out[0] |= 1: a key_hash differs from Long.hashCode(key); out[1] = min(key group + 1) outside
// [kg_lo, kg_hi] when check_range (out[1] must start at ~0)
hipError_t launch_check_keys(int64_t n, const int64_t* key, const int32_t* key_hash, int32_t max_p, int32_t kg_lo,
                             int32_t kg_hi, int check_range, unsigned long long* out, hipStream_t s);
// Stable single-pass partition into per-owner regions of capacity cap (n <= cap, p <=
// kPartRegionMaxOwners): owner q's packed words at packed_out + q * cap, its other records at
// the columns + q * cap; counts as launch_partition's.  scratch: partition_scratch_bytes(n, nd).
constexpr int32_t kPartRegionMaxOwners = 16;
hipError_t launch_partition_regions(int64_t n, const int64_t* key, const int32_t* key_hash, const int64_t* ts,
                                    const int64_t* val, int32_t max_p, int32_t p, int64_t cap, int64_t* key_out,
                                    int64_t* ts_out, int64_t* val_out, int32_t* hash_out, const PackGeom* pack,
                                    uint64_t* packed_out, int64_t* counts, void* scratch, hipStream_t s,
                                    int turn = -1, int32_t nd_max = 0, int unstable = 0);
// turn >= 0 (a caller launching repeatedly on one stream, alternating turn): scratch of
// partition_regions_scratch_bytes(cap, nd_max), zeroed once at allocation; each launch zeroes
// the half the next one uses (no memset per launch).  turn < 0: a memset of this launch's words.
int64_t partition_regions_scratch_bytes(int64_t cap, int32_t nd);
// Stable partition by owner.  pack (enabled): 2p buckets -- 2q: q's packed words in
// packed_out, 2q + 1: q's other records in the columns -- at positions of one numbering;
// counts[2q], counts[2q + 1] their sizes.
hipError_t launch_partition(int64_t n, const int64_t* key, const int32_t* key_hash, const int64_t* ts,
                            const int64_t* val, int32_t max_p, int32_t p, int64_t* key_out,
                            int64_t* ts_out, int64_t* val_out, int64_t* counts, void* scratch,
                            hipStream_t s, int32_t* hash_out = nullptr, const PackGeom* pack = nullptr,
                            uint64_t* packed_out = nullptr);
// gw_select.hip: stable select (sel == want) + dictionary lookup (gw_select_lookup_device)
hipError_t launch_select_lookup(int64_t n, const int64_t* sel, int64_t want, const int64_t* idx, const int64_t* dict,
                                int64_t dict_n, const int64_t* ts, int64_t* key_out, int64_t* ts_out, void* scratch,
                                hipStream_t s);
size_t select_lookup_scratch_bytes(int64_t n);
hipError_t launch_unpack(int64_t n, const uint64_t* w, const PackGeom& g, int64_t* key, int64_t* ts, int64_t* val,
                         hipStream_t s);

// Key -> Java hashCode of the keys a handle was fed with a key_hash column (String,
// Integer, ... keys mapped to int64 ids by the caller).  The heap backend files a key's
// state under the key group of key.hashCode() (KeyGroupRangeAssignment.java:63-66), so a
// snapshot needs the hash of every key holding state.  Open addressing, linear probing;
// key[cap] / hash[cap] hold the key INT64_MIN (key[cap] = 1 once present, else 0).
struct KeyHashMap {
    int64_t* key = nullptr;
    int32_t* hash = nullptr;
    int64_t cap = 0;  // power of two; 0: no map yet
};
// Insert (key, hash) pairs (first hash wins); out[0] += keys inserted.  A second launch
// with verify = 1 counts in out[1] the records whose hash differs from the stored one.
hipError_t launch_khmap_insert(const KeyHashMap& m, int64_t n, const int64_t* key, const int32_t* hash, int verify,
                               unsigned long long* out, hipStream_t s);
// p[0..n) = v
hipError_t launch_fill64(int64_t* p, int64_t n, int64_t v, hipStream_t s);
// keyBy exchange message per peer q: msg[4q..4q+3] = (records, wm, cols, packed records);
// packed: counts holds 2 buckets per peer (packed, other)
// (zeroes the counts it read: the unstable region partition adds into them)
hipError_t launch_exchange_message(int64_t* counts, int32_t p, int64_t wm, int64_t cols, int packed,
                                   int64_t* msg, hipStream_t s);
// Every entry of `from` into the empty map `to`.
hipError_t launch_khmap_rehash(const KeyHashMap& from, const KeyHashMap& to, hipStream_t s);

}  // namespace gw
