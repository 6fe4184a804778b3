// gw_kernels.h — kernel argument blocks and launcher declarations (host <-> device).
#pragma once
#include "gw_device.h"

namespace gw {

struct IngestArgs {
    const int64_t* key;
    const int64_t* ts;
    const int64_t* val;
    int64_t n;
    int64_t t_late;     // first non-late timestamp (start of the first unfired window)
    int64_t p_late;     // its pane index
    uint64_t delta;     // ring base pane B - p_late (>= 0)
    UDiv64 div;         // division by the pane width g
    int32_t b_pos;      // B mod R
    int32_t late_exact; // 0: t_late was clamped at Long.MIN_VALUE (then ts < t_late is a range error)
    TableView t;
    int64_t* d_key;     // deferred list (append at st->n_deferred)
    int64_t* d_pane;
    int64_t* d_a0;
    int64_t* d_a1;
    DevStatus* st;
};

struct MergeArgs {
    const int64_t* i_key;
    const int64_t* i_pane;
    const int64_t* i_a0;
    const int64_t* i_a1;
    int64_t n;
    int64_t b;          // ring base pane
    int32_t b_pos;
    TableView t;
    int64_t* d_key;     // entries still outside the ring (append at st->n_deferred)
    int64_t* d_pane;
    int64_t* d_a0;
    int64_t* d_a1;
    DevStatus* st;
};

struct FireArgs {
    TableView t;
    int32_t nwin;
    int64_t start0;     // start of the first window fired in this pass
    int64_t slide;
    int64_t size;
    uint64_t rmask;     // ring positions retired after this pass
    uint64_t wmask[kMaxRing];
    int64_t* o_key;
    int64_t* o_start;
    int64_t* o_end;
    int64_t* o_res;
    DevStatus* st;
};

struct EvictArgs {
    TableView t;
    uint64_t emask;
    int64_t pane_of_pos[kMaxRing];
    int64_t* d_key;
    int64_t* d_pane;
    int64_t* d_a0;
    int64_t* d_a1;
    DevStatus* st;
};

hipError_t launch_table_init(const TableView& t, hipStream_t s);
hipError_t launch_ingest(const IngestArgs& a, bool preagg, int unroll, hipStream_t s);
hipError_t launch_merge_deferred(const MergeArgs& a, hipStream_t s);
hipError_t launch_deferred_min(const int64_t* pane, int64_t n, DevStatus* st, hipStream_t s);
hipError_t launch_fire(const FireArgs& a, hipStream_t s);
hipError_t launch_evict(const EvictArgs& a, hipStream_t s);
hipError_t launch_rehash(const TableView& o, const TableView& n, DevStatus* st, hipStream_t s);
hipError_t launch_status_set(DevStatus* st, int word, unsigned long long v, int shard_field, hipStream_t s);
hipError_t launch_count_live(const TableView& t, unsigned long long* out, hipStream_t s);

// key groups / exchange (gw_keygroups.hip)
hipError_t launch_key_groups(int64_t n, const int64_t* key, const int32_t* key_hash, int32_t max_p,
                             int32_t p, int32_t* kg, int32_t* owner, hipStream_t s);
int64_t partition_scratch_bytes(int64_t n, int32_t p);
hipError_t launch_partition(int64_t n, const int64_t* key, const int32_t* key_hash, const int64_t* ts,
                            const int64_t* val, int32_t max_p, int32_t p, int64_t* key_out,
                            int64_t* ts_out, int64_t* val_out, int64_t* counts, void* scratch,
                            hipStream_t s);

}  // namespace gw
