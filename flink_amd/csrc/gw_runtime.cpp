// gw_runtime.cpp — host orchestration behind the C ABI of include/gpuwin.h.
//
// One gw_handle = one keyed window operator subtask (Flink: one WindowOperator
// instance on one mailbox thread, RS/runtime/tasks/mailbox/MailboxProcessor.java:45-49).
// Calls on a handle are serialised by the caller; the handle owns its HIP stream,
// its HBM state table and every device buffer.  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <functional>
#include <map>
#include <set>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <tuple>
#include <vector>
#include <mutex>

#include "gw_first.h"
#include "gw_kernels.h"
#include "gw_netbuf.h"
#include "gw_session.h"
#include "gw_sort.h"

using namespace gw;

namespace {

thread_local std::string g_create_error;

constexpr int64_t kMaxIngest = (int64_t)1 << 30;
constexpr uint32_t kSnapMaxVersion = 4;  // gw_handle::SnapHeader versions
constexpr int64_t kSnapKeyHashes = 1;    // SnapHeader::flags
constexpr int64_t kSnapFirstElement = 2; // SnapHeader::flags: v4 entries end with the first element's payload

// Host-time profile of the ingest path (GW_HOST_PROFILE=1: printed by gw_destroy).
struct HostProf {
    bool on = getenv("GW_HOST_PROFILE") != nullptr;
    double t[16] = {};
    int64_t n[16] = {};
    std::chrono::steady_clock::time_point last;
    void mark() { if (on) last = std::chrono::steady_clock::now(); }
    void lap(int i) {
        if (!on) return;
        auto now = std::chrono::steady_clock::now();
        t[i] += std::chrono::duration<double, std::micro>(now - last).count();
        n[i]++;
        last = now;
    }
    void dump() {
        if (!on) return;
        static const char* names[16] = {"prep", "launch", "status-enqueue", "status-wait", "absorb", "api-entry",
                                        "ov_finalize", "refresh", "grow", "deferred", "args", "path-flush",
                                        "region", "fmt", "advance", "-"};
        for (int i = 0; i < 16; ++i)
            if (n[i]) fprintf(stderr, "[gw host] %-15s %8.2f us x %lld\n", names[i], t[i] / n[i], (long long)n[i]);
    }
};

typedef __int128 i128;

i128 floor_div(i128 a, i128 b) {  // b > 0
    i128 q = a / b;
    if ((a % b) != 0 && a < 0) --q;
    return q;
}
i128 floor_mod(i128 a, i128 b) { return a - floor_div(a, b) * b; }
int64_t gcd64(int64_t a, int64_t b) {
    while (b) { int64_t t = a % b; a = b; b = t; }
    return a;
}
bool fits64(i128 v) { return v >= (i128)INT64_MIN && v <= (i128)INT64_MAX; }

UDiv64 make_udiv(uint64_t d) {
    UDiv64 r{};
    if (d == 1) { r.mode = 1; return r; }
    unsigned l = 0;
    while (l < 64 && (1ull << l) < d) ++l;  // l = ceil(log2 d), d >= 2 -> l >= 1
    unsigned __int128 two_l = (unsigned __int128)1 << l;
    unsigned __int128 m = (((two_l - d) << 64) / d) + 1;
    r.magic = (uint64_t)m;
    r.shift = l - 1;
    r.mode = 0;
    return r;
}

// Host copy into pinned staging, split over threads for large columns (one thread's memcpy
// is well below the PCIe rate the H2D copy behind it reaches).
void par_memcpy(void* dst, const void* src, size_t bytes) {
    constexpr size_t kPer = (size_t)32 << 20;
    const int nt = (int)std::min<size_t>(8, bytes / kPer);
    if (nt <= 1) { memcpy(dst, src, bytes); return; }
    std::vector<std::thread> th;
    const size_t part = (bytes / nt + 63) & ~(size_t)63;
    for (int i = 0; i < nt; ++i) {
        const size_t lo = (size_t)i * part;
        if (lo >= bytes) break;
        const size_t len = std::min(part, bytes - lo);
        th.emplace_back([=] { memcpy((char*)dst + lo, (const char*)src + lo, len); });
    }
    for (auto& t : th) t.join();
}

// Several host copies at once, split evenly over up to 8 threads (the pieces of one drain chunk).
void par_copy_multi(const std::vector<std::tuple<void*, const void*, size_t>>& parts) {
    size_t total = 0;
    for (auto& p : parts) total += std::get<2>(p);
    const int nt = (int)std::min<size_t>(8, total / ((size_t)1 << 20));
    if (nt <= 1) {
        for (auto& p : parts) memcpy(std::get<0>(p), std::get<1>(p), std::get<2>(p));
        return;
    }
    const size_t share = (total + nt - 1) / nt;
    std::vector<std::thread> th;
    size_t pi = 0, po = 0;  // next part, offset in it
    for (int t = 0; t < nt && pi < parts.size(); ++t) {
        std::vector<std::tuple<char*, const char*, size_t>> mine;
        size_t left = share;
        while (left && pi < parts.size()) {
            const size_t len = std::min(left, std::get<2>(parts[pi]) - po);
            mine.emplace_back((char*)std::get<0>(parts[pi]) + po, (const char*)std::get<1>(parts[pi]) + po, len);
            left -= len;
            po += len;
            if (po == std::get<2>(parts[pi])) { ++pi; po = 0; }
        }
        th.emplace_back([mine] { for (auto& m : mine) memcpy(std::get<0>(m), std::get<1>(m), std::get<2>(m)); });
    }
    for (auto& t : th) t.join();
}

struct KernelTimer {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
    double total_ms = 0, last_ms = 0;
    int64_t launches = 0;
    std::pair<hipEvent_t, hipEvent_t> get() {
        if (!pool.empty()) { auto p = pool.back(); pool.pop_back(); return p; }
        std::pair<hipEvent_t, hipEvent_t> p;
        hipEventCreate(&p.first);
        hipEventCreate(&p.second);
        return p;
    }
    void resolve() {  // stream already synchronised
        for (auto& p : pending) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
                total_ms += ms;
                last_ms = ms;
                launches++;
            }
            pool.push_back(p);
        }
        pending.clear();
    }
    void drop_last() {  // the last resolved launch did no work (a skipped guarded fire)
        if (launches > 0) {
            launches--;
            total_ms -= last_ms;
        }
    }
    void destroy() {
        for (auto& p : pending) pool.push_back(p);
        for (auto& p : pool) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
        pool.clear();
        pending.clear();
    }
};

}  // namespace

struct gw_handle {
    gw_config cfg{};
    std::string err;
    bool failed = false;
    hipStream_t stream = nullptr;
    // Window-class composite (sliding windows whose pane ring exceeds kMaxRing): J child
    // operators, child j holding the windows k = j (mod J) -- a sliding assigner of slide
    // J * slide and offset offset + j * slide -- on one shared stream; rows gathered by
    // gw_rows_device wait in c_* until drained.
    std::vector<gw_handle*> kids;
    bool shared_stream = false;      // the stream belongs to another handle
    int64_t cls_J = 0, cls_j = 0, cls_slide = 0, cls_off = 0;  // a child's class
    int64_t *c_key = nullptr, *c_start = nullptr, *c_end = nullptr, *c_res = nullptr;
    int64_t c_cap = 0, c_rows = 0, c_head = 0;
    // First-element handle (GW_FLAG_FIRST_ELEMENT, gw_first.hip): kids[0] folds the aggregate,
    // kids[1] the MIN of each record's arrival sequence; the payload log keeps every record's
    // payload (a ring indexed by sequence) until all windows that could hold it are cleaned.
    bool fe = false;
    // GW_FLAG_BY_FIELD (minBy / maxBy): kids[0] alone folds MIN / MAX of the field, the log
    // holds (payload, key, ts, field) per record and each fire picks the element (fe_by_select)
    bool fe_by = false, fe_by_last = false;
    int fe_cols = 1;                                    // log columns of fe_log_cap words each
    int64_t fe_restored_end = 0;                        // sequences below: restored elements
    int64_t fe_seq = 0;                                 // sequence of the next record
    int64_t* fe_log = nullptr;
    int64_t fe_log_cap = 0, fe_log_base = 0;            // live sequences [fe_log_base, fe_seq)
    int64_t* fe_seqbuf = nullptr;
    int64_t fe_seqbuf_cap = 0;
    int64_t* fe_maxts = nullptr;                        // per batch (ring of kFeBatches): largest ts
    struct FeBatch {
        int64_t seq_end;  // sequences of the batch end here
        int64_t slot;     // its max timestamp in fe_maxts[slot] until fetched
        int64_t max_ts;   // fetched max timestamp
        bool known;
    };
    std::vector<FeBatch> fe_batches;  // not yet released, in arrival order
    int64_t fe_wm = INT64_MIN;        // the last watermark (release decisions)
    int64_t fe_batch_no = 0;
    int64_t* c_pay = nullptr;
    void* fe_scratch = nullptr;
    size_t fe_scratch_bytes = 0;
    int32_t* fe_bad = nullptr;
    static constexpr int64_t kFeBatches = 1 << 16;
    hipEvent_t ev_in = nullptr, ev_out = nullptr;  // gw_ingest_device ordering with the producer stream

    // network-buffer ingest (gw_ingest_serialized*): grow-only device scratch, decoded
    // columns, watermark list, pinned status and staging for host bytes
    void* nb_scratch = nullptr;
    int64_t nb_scratch_cap = 0;
    int64_t* nb_cols = nullptr;  // key | ts | value, nb_rec_cap each
    int64_t nb_rec_cap = 0;
    int64_t* nb_wm = nullptr;    // position | value, nb_wm_cap each
    int64_t nb_wm_cap = 0;
    NbStatus* d_nbst = nullptr;
    NbStatus* h_nbst = nullptr;  // pinned
    int64_t* h_nbwm = nullptr;   // pinned, 2 * kNbWmHost
    uint8_t* h_nbbytes = nullptr;
    uint8_t* d_nbbytes = nullptr;
    int64_t nb_bytes_cap = 0;
    static constexpr int64_t kNbWmHost = 4096;
    bool session = false;

    // pane geometry
    int64_t g = 1, m = 1, n = 1;
    int64_t gap_size = 0;  // size < slide: panes of width slide, records past `size` into one are skipped
    int R = 2;
    UDiv64 div{};

    // state table (region-major SoA, gw_kernels.h)
    PaneTable tv{};
    size_t table_bytes = 0;

    // Buffer of P1 tiles (k_rgn_p1) and the flush scratch (k_rgn_plan*, k_rgn_p2), sized
    // in 4096-record tiles; every array below holds buf_cap tiles' worth.
    int64_t* e_col[6] = {};         // e_key e_a0 e_a1 (P2 output) p1_key p1_a0 p1_a1 (P1 output)
    uint8_t* e_pos[2] = {};         // e_pos p1_pos
    uint32_t* p1_row = nullptr;     // [tile][kPartBuckets]
    uint32_t* p2_desc = nullptr;    // [bucket][tile]
    int64_t* p2_off = nullptr;      // [blocks + 1], blocks = buckets x groups <= 2 tiles + kPartBuckets
    int64_t* p2_roff = nullptr;
    int64_t* rbeg = nullptr;        // [kPartBuckets + 1] rounds | [kPartBuckets + 1] records (bk_off)
    uint32_t* r_row = nullptr;      // [rounds][kPartBuckets], rounds <= tiles + blocks
    int64_t* r_base = nullptr;      // [rounds]
    int64_t buf_cap = 0;            // tiles
    uint64_t stale_pos = 0;         // ring positions retired lazily, not yet cleaned (lazy_retire)
    static int64_t max_blocks(int64_t tiles) { return 2 * tiles + kPartBuckets + 1; }
    static int64_t max_rounds(int64_t tiles) { return tiles + max_blocks(tiles); }

    // buffered region ingest: P1 segments waiting for P2 + apply
    int nseg = 0;
    int64_t buf_tiles = 0;          // tiles used by the waiting segments
    uint64_t buf_fresh = 0;         // ring positions holding only identities at buffer start
    int buf_fmt = 0;                // record format of the waiting segments (fixed per window):
                                    // 0 wide, 1 compact, 2 narrow (gw_pane.hip kFmt*)
    int64_t buf_recs = 0;           // records of the waiting segments
    bool cmp_off = false;           // compact records turned off: too many values beyond 32 bits
    bool nar_off = false;           // narrow records turned off: too many keys / values beyond them
    int64_t buf_limit = (int64_t)1 << 27;  // records (GW_BUFFER_RECORDS)
    // nar2 carry: a fire's flush applies only the ring positions the fire needs
    // and leaves the newer ones in its P2 output, which the next flush applies from there.  Two
    // P2 output sets (key words, round rows, round bases, rbeg | bk_off) used in turn: eset is
    // the one the next P2 writes; while carry_on, set eset ^ 1 holds carry_mask's positions.
    int64_t* e2_key = nullptr;
    uint32_t* r_row2 = nullptr;
    int64_t* r_base2 = nullptr;
    int64_t* rbeg2 = nullptr;
    int64_t e2_cap = 0;             // tiles
    int eset = 0;
    bool carry_on = false;
    uint64_t carry_mask = 0;
    int64_t* eset_key(int s) const { return s ? e2_key : e_col[0]; }
    uint32_t* eset_row(int s) const { return s ? r_row2 : r_row; }
    int64_t* eset_base(int s) const { return s ? r_base2 : r_base; }
    int64_t* eset_rbeg(int s) const { return s ? rbeg2 : rbeg; }

    // allowed lateness > 0 (tumbling / sliding): late records of fired, not yet cleaned
    // windows wait on the re-fire list until the next watermark (process_refire)
    int64_t* rf[5] = {};            // key, pane, a0, a1, arrival number
    int64_t rf_cap = 0;
    int64_t rf_bound = 0;           // records ingested since the list was last processed
    int64_t seq_ctr = 0;            // arrival number of the next record
    int64_t rf_seq_base = 0;        // arrival number at the last processing
    void* rf_sort = nullptr;        // sort keys / payloads / scratch
    int64_t rf_sort_bytes = 0;

    // late-data side output (GW_FLAG_LATE_SIDE_OUTPUT): key | ts | value, [lo_head, n_late_out) pending
    int64_t* lo_buf[3] = {nullptr, nullptr, nullptr};
    int64_t lo_cap = 0, lo_head = 0;
    int64_t lo_bound = 0;  // records ingested since the buffer was last emptied (bounds n_late_out)
    bool late_out() const { return (cfg.flags & GW_FLAG_LATE_SIDE_OUTPUT) != 0; }

    // event-time state
    int64_t wm = INT64_MIN;
    i128 fired_k = 0;  // first window index not yet fired
    i128 B = 0;        // ring base pane
    uint64_t occ = 0;  // ring positions that may hold data

    // deferred lists (double-buffered)
    int64_t* dk[2] = {nullptr, nullptr};
    int64_t* dp[2] = {nullptr, nullptr};
    int64_t* da0[2] = {nullptr, nullptr};
    int64_t* da1[2] = {nullptr, nullptr};
    int64_t def_cap = 0;
    int cur = 0;

    // Host-ingest staging (gw_ingest, gw_stage_*).  Pinned host slots (key | ts | value columns
    // of slot_cap records, then the int32 key hashes) that a caller fills in place (a JVM writes
    // its records straight into them) or gw_ingest copies into; each batch goes over PCIe on a
    // copy stream into one of three device staging buffers used in turn, so the H2D of batches
    // b+1 and b+2 runs while batch b is aggregated, fired and drained.  A slot is refilled only after its H2D (ev_slot); a
    // device buffer is overwritten only after the ingest that read it (ev_dread).
    std::vector<int64_t*> h_slot;
    std::vector<hipEvent_t> ev_slot;
    std::vector<bool> slot_used;
    int64_t slot_cap = 0;
    int stage_next = 0;             // gw_ingest's next slot (of the first two)
    static constexpr int kStageBufs = 3;  // device buffers: up to two batches sent ahead of the ingest
    int64_t* d_stage2[kStageBufs] = {};
    hipEvent_t ev_dread[kStageBufs] = {};
    bool dread_valid[kStageBufs] = {};
    int dturn = 0;                  // the device buffer the next staged ingest reads
    int send_turn = 0;              // the device buffer the next H2D fills
    // a slot already sent ahead (gw_stage_send) into device buffer t, not yet ingested
    bool pre_valid[kStageBufs] = {};
    bool slots_out = false;  // gw_stage_columns handed out pointers into the pinned slots
    int pre_slot[kStageBufs] = {-1, -1, -1};
    int64_t pre_n[kStageBufs] = {};
    int pre_cols[kStageBufs] = {};
    hipStream_t cstream = nullptr;
    // staged H2D split over extra copy streams (GW_STAGE_STREAMS > 1): several DMA queues
    // in flight, joined back into cstream by events
    std::vector<hipStream_t> cx;
    std::vector<hipEvent_t> cx_ev;
    hipEvent_t ev_fork = nullptr;

    // output rows (device SoA), [rows_head, st.rows) pending
    int64_t* o_key = nullptr;
    int64_t* o_start = nullptr;
    int64_t* o_end = nullptr;
    int64_t* o_res = nullptr;
    int64_t o_cap = 0;
    int64_t rows_head = 0;

    // status
    DevStatus* d_st = nullptr;
    DevStatus* h_st = nullptr;
    unsigned long long* d_tmp = nullptr;

    gw_stats stats{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -1};
    bool timing = false;
    KernelTimer t_ingest, t_fire, t_apply;
    int64_t timing_every = 1, timing_ctr = 0;  // region pass 1: time one launch in timing_every
    HostProf hp;
    // gw_ingest_packed_device: the batch's records [pk_from, n) are packed exchange words that
    // the region P1 decodes itself; other paths get them unpacked into pk_stage first
    const uint64_t* pk_w = nullptr;
    int64_t pk_from = 0;
    gw_pack_geom pk_g{};
    int64_t* pk_stage = nullptr;
    int64_t pk_stage_cap = 0;

    SessionState* sess = nullptr;
    // key checks (gw_ingest* with key_hash, GW_FLAG_CHECK_KEY_GROUPS): device words, see k_check_keys
    unsigned long long* d_chk = nullptr;
    bool foreign_hash = false;  // a key_hash differed from Long.hashCode(key) (keys are caller ids)
    int ingest_unroll = 2;  // records per thread per iteration of k_ingest (GW_INGEST_UNROLL)
    int64_t region_min_batch = 1 << 16;  // smallest batch for the region path (GW_REGION_MIN_BATCH)
    // records ingested since the last fire, and over the last fire cycle: the region path
    // buffers batches until a fire, so its state pass amortises over a whole cycle
    int64_t recs_since_fire = 0, recs_per_fire = 0;

    int fail(int code, const char* fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        err = buf;
        if (code == GW_E_DEVICE || code == GW_E_NO_TIMESTAMP || code == GW_E_RANGE) failed = true;
        return code;
    }
#define HIPCHECK(x)                                                                                  \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) return fail(GW_E_DEVICE, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

    bool dirty = true;  // device counters changed since the last refresh()

    // Lazy status (buffered region P1 only): a one-workgroup kernel behind each P1 launch
    // (k_publish_status, same stream) writes the status into a pinned host slot and
    // stamps it with the launch's sequence number.  The host reads the slot of batch b
    // while batch b + 1 is already queued, so the GPU does not wait for the host between watermark batches and
    // the stream carries no event or copy between them.  h_st then lags by the last
    // batches (`lazy`): decisions that need exact counters call refresh().
    static constexpr int kAsync = 3;  // slots in flight: absorb the one 2 batches old
    DevStatus* h_st_async[kAsync] = {};
    uint64_t async_seq[kAsync] = {};
    uint64_t pub_ctr = 0;
    bool async_pending[kAsync] = {};
    uint64_t async_gen[kAsync] = {};
    int64_t async_recs[kAsync] = {};    // records of the batch each copy follows
    uint64_t hgen = 0;        // host writes to the status (a snapshot older than one is stale)
    int async_slot = 0;
    // gw_clear_rows on the host only: the device's row cursor is zeroed by the next launch that
    // emits rows (the fast fire's guard, or a status write before any other fire); until then
    // every status the host reads has its row count taken as 0
    bool rows_reset_pending = false;
    bool occ_zeroed = false;  // batch_occ (d_tmp[1]) zeroed behind the last flush, no pass 1 since
    bool lazy = false;        // launches since the last exact status: region P1 only
    int64_t lazy_recs = 0;    // records of those launches (bound on their deferred entries)

    int refresh() {
        HIPCHECK(hipMemcpyAsync(h_st, d_st, sizeof(DevStatus), hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        for (auto& p : async_pending) p = false;  // older than this copy
        lazy = false;
        lazy_recs = 0;
        dirty = false;
        if (timing) { t_ingest.resolve(); t_fire.resolve(); t_apply.resolve(); }
        return absorb();
    }
    // Arm the status slot the next buffered P1 publishes into.
    void arm_status(IngestArgs& a) {
        const int s = async_slot;
        volatile uint64_t* tag = (volatile uint64_t*)&h_st_async[s]->pad[kPubSeqWord];
        *tag = 0;
        a.st_host = h_st_async[s];
        a.st_seq = async_seq[s] = ++pub_ctr;
    }
    // Wait until slot o carries its launch's stamp (the P1 has finished publishing).
    // The tag is polled in host memory; the stream is queried only after the wait has lasted
    // 1 ms, then every 1 ms (a failed or finished stream whose P1 never published): each
    // hipStreamQuery on a busy stream put a ~5-us gap between the queued P1 launches
    // (profiles/r6/gaps/).
    int wait_published(int o) {
        volatile uint64_t* tag = (volatile uint64_t*)&h_st_async[o]->pad[kPubSeqWord];
        auto next_query = std::chrono::steady_clock::time_point::min();
        for (int64_t spin = 0; *tag != async_seq[o]; ++spin) {
            if ((spin & 255) == 255) {
                const auto now = std::chrono::steady_clock::now();
                if (next_query == std::chrono::steady_clock::time_point::min()) {
                    next_query = now + std::chrono::milliseconds(1);
                    continue;
                }
                if (now < next_query) { std::this_thread::yield(); continue; }
                next_query = now + std::chrono::milliseconds(1);
                const hipError_t q = hipStreamQuery(stream);
                if (q == hipSuccess && *tag != async_seq[o])
                    return fail(GW_E_DEVICE, "status slot not published by the finished pass 1");
                if (q != hipSuccess && q != hipErrorNotReady)
                    return fail(GW_E_DEVICE, "pass 1 failed: %s", hipGetErrorString(q));
                std::this_thread::yield();
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        return GW_OK;
    }
    // After a buffered P1 launch: absorb the slot published two launches ago.
    int lazy_status(int64_t nrec) {
        const int s = async_slot;
        hp.lap(1);
        async_pending[s] = true;
        async_gen[s] = hgen;
        async_recs[s] = nrec;
        async_slot = (s + 1) % kAsync;
        lazy = true;
        lazy_recs += nrec;
        const int o = async_slot;  // the oldest slot
        hp.lap(2);
        if (!async_pending[o]) return GW_OK;
        async_pending[o] = false;
        int rc;
        if ((rc = wait_published(o))) return rc;
        hp.lap(3);
        if (async_gen[o] != hgen) return GW_OK;  // the host changed the status since
        memcpy(h_st, h_st_async[o], sizeof(DevStatus));
        // unaccounted for: the absorbed slot's own batch (its P1 published at its start) and
        // every batch after it
        lazy_recs = async_recs[o];
        for (int i = 0; i < kAsync; ++i)
            if (async_pending[i]) lazy_recs += async_recs[i];
        rc = absorb();
        hp.lap(4);
        return rc;
    }
    int absorb() {
        fold_shards(h_st);
        if (rows_reset_pending) h_st->rows = 0;
        if (h_st->flags & GW_DF_NO_TS)
            return fail(GW_E_NO_TIMESTAMP,
                        "Record has Long.MIN_VALUE timestamp (= no timestamp marker). Did you forget to "
                        "call 'DataStream.assignTimestampsAndWatermarks(...)'?");
        if (h_st->flags & GW_DF_RANGE)
            return fail(GW_E_RANGE, "record timestamp/pane outside the supported int64 window range");
        occ = h_st->occ;
        stats.late_dropped = (int64_t)h_st->late;
        stats.live_keys = (int64_t)h_st->used_slots;
        stats.deferred = (int64_t)h_st->n_deferred;
        stats.session_merges = (int64_t)h_st->merges;
        return GW_OK;
    }
    int ensure_fresh() { return dirty || lazy ? refresh() : GW_OK; }
    // Write one scalar status word, ordered on the stream (no host sync).
    int set_field(size_t off, unsigned long long v) {
        hgen++;
        *reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(h_st) + off) = v;
        HIPCHECK(launch_status_set(d_st, (int)(off / 8), v, -1, stream));
        return GW_OK;
    }
    // Zero one field of every counter shard (field index within ShardCtr).
    int zero_shards(int field) {
        hgen++;
        for (int i = 0; i < kShards; ++i) reinterpret_cast<unsigned long long*>(&h_st->sh[i])[field] = 0;
        HIPCHECK(launch_status_set(d_st, 0, 0, field, stream));
        dirty = true;
        return GW_OK;
    }
    int take_occ() { occ = h_st->occ; return GW_OK; }
    // The deferred gw_clear_rows, before a launch that moves the row cursor.
    int rows_reset_now() {
        if (!rows_reset_pending) return GW_OK;
        rows_reset_pending = false;
        return set_field(offsetof(DevStatus, rows), 0);
    }

    // ---------------------------------------------------------------- memory
    // Pane-table load: the table is sized for the expected keys at kTableLoad and grows past
    // kGrowLoad.  The geometry allows any load (regions per bucket need not be a
    // power of two); measured on the headline (profiles/r6/): 0.8 -- 12.6M slots for 10M keys,
    // ~85% of the keys in their home group of 4 slots against 0.93 at 0.6 -- made the apply
    // and the fire slower, so the default stays at 0.6 (8192 regions for 10M keys).
#ifndef GW_TABLE_LOAD
#define GW_TABLE_LOAD 0.6
#endif
    static constexpr double kTableLoad = GW_TABLE_LOAD,
                            kGrowLoad = GW_TABLE_LOAD + 0.1 < 0.88 ? GW_TABLE_LOAD + 0.1 : 0.88;
    // Region-major table: nreg = nsub << rb1 regions of S slots (table_geometry).
    static size_t pane_table_bytes(const PaneTable& t) { return (size_t)(t.nreg + 1) * (size_t)t.region_words * 8; }
    // At least `want` slots: regions of S = 2048 slots (1024 for two-word cells: keys + mask +
    // two pane arrays take ~50 KB of LDS in k_rgn_apply; 1024-slot regions measured slower).  Up
    // to 128 regions: a power of two, single-pass (one pass-1 bucket per region).  Beyond: 2^rb1
    // = 128 (256 past 8192 regions) pass-1 buckets of nsub regions, nsub any even number (a
    // multiple of 4 past 64), so the capacity follows the keys in steps of 1/64 instead of 2x.
    static void table_geometry(PaneTable& t, int64_t want) {
        int64_t S = t.words == 2 ? 1024 : 2048;
        want = std::max<int64_t>(want, 16);
        int64_t nreg_want = (want + S - 1) / S;
        if (nreg_want <= 1) {  // one region of a power of two (>= 16) slots
            S = 16;
            while (S < want) S *= 2;
            nreg_want = 1;
        }
        int l2s = 0;
        while (((int64_t)1 << l2s) < S) ++l2s;
        t.log2S = l2s;
        if (nreg_want <= 128) {
            int l2r = 0;
            while (((int64_t)1 << l2r) < nreg_want) ++l2r;
            t.rb1 = l2r;
            t.nsub = 1;
        } else {
            t.rb1 = nreg_want <= 128 * 64 ? 7 : 8;
            int64_t nsub = (nreg_want + (1 << t.rb1) - 1) >> t.rb1;
            const int64_t q = nsub > 64 ? 4 : 2;  // nar2 super-regions of 2 (4) regions
            nsub = std::min<int64_t>((nsub + q - 1) / q * q, kRgnMaxRegions >> t.rb1);
            t.nsub = (int32_t)nsub;
        }
        t.nreg = (int64_t)t.nsub << t.rb1;
        t.cap = t.nreg << l2s;
    }
    int alloc_table(PaneTable& t, int64_t want) {
        t = tv;
        table_geometry(t, want);
        const int64_t S = pt_S(t);
        t.mask_shift = t.ring <= 8 ? 0 : t.ring <= 16 ? 1 : t.ring <= 32 ? 2 : 3;
        t.region_words = S + pt_mask_words(t) + S * (int64_t)t.ring * t.words;
        HIPCHECK(hipMalloc((void**)&t.base, pane_table_bytes(t)));
        HIPCHECK(launch_table_init(t, stream));
        return GW_OK;
    }
    void free_region() {
        for (void** p : {(void**)&e2_key, (void**)&r_row2, (void**)&r_base2, (void**)&rbeg2}) {
            if (*p) hipFree(*p);
            *p = nullptr;
        }
        e2_cap = 0;
        eset = 0;
        for (auto& p : e_col) { if (p) hipFree(p); p = nullptr; }
        for (auto& p : e_pos) { if (p) hipFree(p); p = nullptr; }
        for (void** p : {(void**)&p1_row, (void**)&p2_desc, (void**)&p2_off, (void**)&p2_roff, (void**)&r_row,
                         (void**)&r_base}) {
            if (*p) hipFree(*p);
            *p = nullptr;
        }
        buf_cap = 0;
    }
    // Region buffer of >= need tiles (re-allocated to `want` tiles when too small; only
    // with no segment waiting).
    int ensure_region(int64_t need, int64_t want) {
        if (!rbeg) HIPCHECK(hipMalloc((void**)&rbeg, (size_t)2 * (kPartBuckets + 1) * 8));  // rbeg | bk_off
        if (need <= buf_cap) return GW_OK;
        if (carry_on) {  // the carried records live in the buffers about to be re-allocated
            int rc = flush_buffer();
            if (rc) return rc;
        }
        if (nseg) return fail(GW_E_STATE, "internal: region buffer re-allocated with %d segments waiting", nseg);
        const int64_t cap = std::max(need, want);
        const size_t recs = (size_t)cap * kPartTile;
        hipStreamSynchronize(stream);
        free_region();
        for (int i = 0; i < 6; ++i) {
            if ((i == 2 || i == 5) && tv.words != 2) continue;  // a1 only for AVG
            HIPCHECK(hipMalloc((void**)&e_col[i], recs * 8));
        }
        for (auto& p : e_pos) HIPCHECK(hipMalloc((void**)&p, recs));
        HIPCHECK(hipMalloc((void**)&p1_row, (size_t)cap * kPartBuckets * 4));
        HIPCHECK(hipMalloc((void**)&p2_desc, (size_t)cap * kPartBuckets * 4));
        HIPCHECK(hipMalloc((void**)&p2_off, (size_t)max_blocks(cap) * 8));
        HIPCHECK(hipMalloc((void**)&p2_roff, (size_t)max_blocks(cap) * 8));
        HIPCHECK(hipMalloc((void**)&r_row, (size_t)max_rounds(cap) * kPartBuckets * 4));
        HIPCHECK(hipMalloc((void**)&r_base, (size_t)max_rounds(cap) * 8));
        buf_cap = cap;
        return GW_OK;
    }
    // The second P2 output set (nar2 carry), as large as the first.
    int ensure_eset2() {
        if (e2_cap == buf_cap && e2_key) return GW_OK;
        for (void** p : {(void**)&e2_key, (void**)&r_row2, (void**)&r_base2, (void**)&rbeg2}) {
            if (*p) hipFree(*p);
            *p = nullptr;
        }
        const size_t recs = (size_t)buf_cap * kPartTile;
        HIPCHECK(hipMalloc((void**)&e2_key, recs * 8));
        HIPCHECK(hipMalloc((void**)&r_row2, (size_t)max_rounds(buf_cap) * kPartBuckets * 4));
        HIPCHECK(hipMalloc((void**)&r_base2, (size_t)max_rounds(buf_cap) * 8));
        HIPCHECK(hipMalloc((void**)&rbeg2, (size_t)2 * (kPartBuckets + 1) * 8));
        e2_cap = buf_cap;
        return GW_OK;
    }
    int ensure_deferred(int64_t need) {
        if (need <= def_cap) return GW_OK;
        // 1.5x: a reallocation costs a sync, ~1 ms of hipMalloc and a copy (measured on the Q7
        // stream, whose few values beyond the narrow record's 28 bits defer and grow the list
        // over a fire cycle), so the list grows in few steps
        int64_t nc = std::max<int64_t>(need + need / 2, 1 << 16);
        for (int b = 0; b < 2; ++b) {
            int64_t* nk; int64_t* np; int64_t* n0; int64_t* n1;
            HIPCHECK(hipMalloc((void**)&nk, nc * 8));
            HIPCHECK(hipMalloc((void**)&np, nc * 8));
            HIPCHECK(hipMalloc((void**)&n0, nc * 8));
            HIPCHECK(hipMalloc((void**)&n1, nc * 8));
            if (dk[b] && b == cur) {
                // a lagging status does not know the last batch's entries: copy them all
                const int64_t used = lazy ? def_cap : (int64_t)h_st->n_deferred;
                if (used) {
                    HIPCHECK(hipMemcpyAsync(nk, dk[b], used * 8, hipMemcpyDeviceToDevice, stream));
                    HIPCHECK(hipMemcpyAsync(np, dp[b], used * 8, hipMemcpyDeviceToDevice, stream));
                    HIPCHECK(hipMemcpyAsync(n0, da0[b], used * 8, hipMemcpyDeviceToDevice, stream));
                    HIPCHECK(hipMemcpyAsync(n1, da1[b], used * 8, hipMemcpyDeviceToDevice, stream));
                }
            }
            if (dk[b]) {
                hipStreamSynchronize(stream);
                hipFree(dk[b]); hipFree(dp[b]); hipFree(da0[b]); hipFree(da1[b]);
            }
            dk[b] = nk; dp[b] = np; da0[b] = n0; da1[b] = n1;
        }
        def_cap = nc;
        return GW_OK;
    }
    int ensure_output(int64_t need) {  // need = total rows (pending + new)
        if (need <= o_cap) return GW_OK;
        int64_t nc = std::max<int64_t>(need + need / 4, 1 << 16);
        int64_t* nb[4];
        for (int i = 0; i < 4; ++i) HIPCHECK(hipMalloc((void**)&nb[i], nc * 8));
        const int64_t used = (int64_t)h_st->rows;
        int64_t* old[4] = {o_key, o_start, o_end, o_res};
        for (int i = 0; i < 4; ++i) {
            if (old[i]) {
                if (used) HIPCHECK(hipMemcpyAsync(nb[i], old[i], used * 8, hipMemcpyDeviceToDevice, stream));
                hipStreamSynchronize(stream);
                hipFree(old[i]);
            }
        }
        o_key = nb[0]; o_start = nb[1]; o_end = nb[2]; o_res = nb[3];
        o_cap = nc;
        return GW_OK;
    }
    void free_stage() {
        if (cstream) hipStreamSynchronize(cstream);
        hipStreamSynchronize(stream);
        for (size_t i = 0; i < h_slot.size(); ++i) {
            if (h_slot[i]) hipHostFree(h_slot[i]);
            if (ev_slot[i]) hipEventDestroy(ev_slot[i]);
        }
        h_slot.clear();
        ev_slot.clear();
        slot_used.clear();
        for (int t = 0; t < kStageBufs; ++t) {
            if (d_stage2[t]) hipFree(d_stage2[t]);
            d_stage2[t] = nullptr;
            dread_valid[t] = false;
            pre_valid[t] = false;
        }
        dturn = send_turn = 0;
        slot_cap = 0;
    }
    // `slots` pinned slots of >= n records each (and the two device buffers of that size).
    int ensure_stage(int64_t n, int slots = 2) {
        if (n <= slot_cap && (int)h_slot.size() >= slots) return GW_OK;
        // reallocating frees the slots: not while batches sent ahead wait in the device
        // buffers, nor once a caller holds pointers into them (JVM direct ByteBuffers)
        for (int t = 0; t < kStageBufs; ++t)
            if (pre_valid[t])
                return fail(GW_E_STATE, "staging: %lld records need larger staging buffers while batches sent "
                                        "ahead (gw_stage_send) are not ingested yet", (long long)n);
        if (slots_out)
            return fail(GW_E_STATE, "staging: %lld records (%d slots) need larger pinned slots than gw_stage_alloc "
                                    "made (%lld records, %d slots), and gw_stage_columns handed those out",
                        (long long)n, slots, (long long)slot_cap, (int)h_slot.size());
        const int64_t cap = std::max(n, slot_cap);
        const int ns = std::max(slots, (int)h_slot.size());
        free_stage();
        if (!cstream) HIPCHECK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
        if (cx.empty()) {
            const char* e = getenv("GW_STAGE_STREAMS");
            const int ncx = e ? std::min(8, std::max(1, atoi(e))) : 1;
            if (ncx > 1) {
                HIPCHECK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
                cx.assign(ncx, nullptr);
                cx_ev.assign(ncx, nullptr);
                for (int i = 0; i < ncx; ++i) {
                    HIPCHECK(hipStreamCreateWithFlags(&cx[i], hipStreamNonBlocking));
                    HIPCHECK(hipEventCreateWithFlags(&cx_ev[i], hipEventDisableTiming));
                }
            }
        }
        for (int t = 0; t < kStageBufs; ++t) {
            if (!ev_dread[t]) HIPCHECK(hipEventCreateWithFlags(&ev_dread[t], hipEventDisableTiming));
            HIPCHECK(hipMalloc((void**)&d_stage2[t], (size_t)cap * 28));
        }
        h_slot.assign(ns, nullptr);
        ev_slot.assign(ns, nullptr);
        slot_used.assign(ns, false);
        for (int i = 0; i < ns; ++i) {
            HIPCHECK(hipHostMalloc((void**)&h_slot[i], (size_t)cap * 28, hipHostMallocDefault));
            HIPCHECK(hipEventCreateWithFlags(&ev_slot[i], hipEventDisableTiming));
        }
        slot_cap = cap;
        return GW_OK;
    }
    // Fired rows to caller memory (any host memory, e.g. a JVM direct ByteBuffer): large
    // drains go through two pinned bounce chunks -- the D2H of chunk j+1 runs while chunk j is
    // copied out by several threads -- instead of one pageable copy per column.
    int64_t* h_bounce = nullptr;
    hipEvent_t ev_bounce[2] = {nullptr, nullptr};
    static constexpr int64_t kBounceRows = (int64_t)1 << 21;  // per chunk and column (16 MB)
    static bool host_pinned(const void* p) {
        hipPointerAttribute_t at;
        if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
            (void)hipGetLastError();  // pageable memory reports an error: clear it
            return false;
        }
        return at.type == hipMemoryTypeHost;
    }
    int drain_to_host(int64_t* const dst[4], const int64_t* const src[4], int64_t c) {
        static const bool direct = [] { const char* v = getenv("GW_DRAIN_BOUNCE"); return v && atoi(v) == 0; }();
        bool pinned = true;  // pinned destinations (page-locked: hipHostMalloc / registered) take the D2H directly
        for (int i = 0; i < 4 && pinned; ++i)
            if (dst[i]) pinned = host_pinned(dst[i]);
#ifdef GW_DEBUG_LOG  // experiment builds only
        fprintf(stderr, "[gw drain] %lld rows, %s\n", (long long)c, direct || pinned || c < kBounceRows / 4 ? (pinned ? "direct (pinned)" : "direct") : "bounce");
#endif
        if (direct || pinned || c < kBounceRows / 4) {
            hipError_t err = hipSuccess;
            for (int i = 0; i < 4 && err == hipSuccess; ++i)
                if (dst[i]) err = hipMemcpyAsync(dst[i], src[i], c * 8, hipMemcpyDeviceToHost, stream);
            if (err == hipSuccess) err = hipStreamSynchronize(stream);
            if (err != hipSuccess) return fail(GW_E_DEVICE, "D2H rows: %s", hipGetErrorString(err));
            return GW_OK;
        }
        if (!h_bounce) {
            HIPCHECK(hipHostMalloc((void**)&h_bounce, (size_t)2 * 4 * kBounceRows * 8, hipHostMallocDefault));
            for (auto& ev : ev_bounce) HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        }
        const int64_t nch = (c + kBounceRows - 1) / kBounceRows;
        auto issue = [&](int64_t j) -> hipError_t {
            const int64_t lo = j * kBounceRows, len = std::min(kBounceRows, c - lo);
            int64_t* b = h_bounce + (j & 1) * 4 * kBounceRows;
            hipError_t err = hipSuccess;
            for (int i = 0; i < 4 && err == hipSuccess; ++i)
                if (dst[i]) err = hipMemcpyAsync(b + i * kBounceRows, src[i] + lo, len * 8, hipMemcpyDeviceToHost, stream);
            return err == hipSuccess ? hipEventRecord(ev_bounce[j & 1], stream) : err;
        };
        hipError_t err = issue(0);
        for (int64_t j = 0; j < nch && err == hipSuccess; ++j) {
            if (j + 1 < nch) err = issue(j + 1);
            if (err == hipSuccess) err = hipEventSynchronize(ev_bounce[j & 1]);
            if (err != hipSuccess) break;
            const int64_t lo = j * kBounceRows, len = std::min(kBounceRows, c - lo);
            const int64_t* b = h_bounce + (j & 1) * 4 * kBounceRows;
            std::vector<std::tuple<void*, const void*, size_t>> parts;
            for (int i = 0; i < 4; ++i)
                if (dst[i]) parts.emplace_back(dst[i] + lo, b + i * kBounceRows, (size_t)len * 8);
            par_copy_multi(parts);
        }
        if (err != hipSuccess) return fail(GW_E_DEVICE, "D2H rows: %s", hipGetErrorString(err));
        return GW_OK;
    }
    // Wait until slot i's last H2D has read it (the caller may write it then).
    int slot_ready(int i) {
        if (slot_used[i]) {
            hipError_t e = hipEventSynchronize(ev_slot[i]);
            if (e != hipSuccess) return fail(GW_E_DEVICE, "staging: %s", hipGetErrorString(e));
        }
        return GW_OK;
    }

    // Re-hash the live slots into a table of `new_cap` slots (drops dead keys).
    int rehash(int64_t new_cap) {
        PaneTable nt;
        int rc = alloc_table(nt, new_cap);
        if (rc) return rc;
        if ((rc = zero_shards(1))) return rc;                          // ins (used slots)
        if (h_st->flags & GW_DF_TABLE_FULL)
            if ((rc = zero_shards(2))) return rc;                      // flags
        HIPCHECK(launch_rehash(tv, nt, d_st, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        HIPCHECK(hipFree(tv.base));
        tv = nt;
        table_bytes = pane_table_bytes(nt);
        stats.rehashes++;
        if ((rc = refresh())) return rc;
        if (h_st->flags & GW_DF_TABLE_FULL) return fail(GW_E_OOM, "state table rehash overflow");
        return ov_attach();  // restored keys without new records are not live slots: re-insert
    }
    int64_t live_count() {
        hipMemsetAsync(d_tmp, 0, 8, stream);
        launch_count_live(tv, d_tmp, stream);
        unsigned long long v = 0;
        hipMemcpyAsync(&h_st->pad[0], d_tmp, 8, hipMemcpyDeviceToHost, stream);
        hipStreamSynchronize(stream);
        v = h_st->pad[0];
        return (int64_t)v;
    }
    // Keep the load factor of the linear-probing table below 0.7.
    int maybe_grow(int64_t incoming) {
        if (nseg || carry_on) {  // waiting segments are bucketed for this table's regions: apply them first
            if (!(h_st->flags & GW_DF_TABLE_FULL) && (double)h_st->used_slots <= kGrowLoad * (double)tv.cap) return GW_OK;
            int rc = flush_buffer();  // refreshes the counters (and may grow by itself)
            if (rc) return rc;
        }
        const int64_t used = (int64_t)h_st->used_slots;
        const bool full = (h_st->flags & GW_DF_TABLE_FULL) != 0;
        if (!full && (double)used <= kGrowLoad * (double)tv.cap) return GW_OK;
        const int64_t live = live_count() + ov_nkeys;
        // parked records that failed to insert are potential new keys
        const int64_t pending = full ? std::max<int64_t>(incoming, (int64_t)h_st->n_deferred) : 0;
        // room for the live keys at the creation load, and at least 1.25x (2x when regions
        // filled up) the current table
        const double floor_x = full ? 2.0 : 1.25;
        const int64_t want = std::max<int64_t>((int64_t)((double)(live + pending) / kTableLoad) + 1,
                                               (int64_t)(floor_x * (double)std::max<int64_t>(tv.cap, 1024)));
        return rehash(want);
    }

    // ---------------------------------------------------------------- pane mode
    int64_t pos_of(i128 pane) const { return (int64_t)floor_mod(pane, R); }

    int merge_deferred() {
        int rc;
        if ((nseg || carry_on) && (rc = flush_buffer())) return rc;  // the merge writes the table directly
        const int64_t nin = (int64_t)h_st->n_deferred;
        if (nin == 0) return GW_OK;
        for (int attempt = 0; attempt < 8; ++attempt) {
            if ((rc = ensure_deferred(nin))) return rc;
            if ((rc = set_field(offsetof(DevStatus, n_deferred), 0))) return rc;
            MergeArgs a{};
            a.i_key = dk[cur]; a.i_pane = dp[cur]; a.i_a0 = da0[cur]; a.i_a1 = da1[cur];
            a.n = nin;
            a.b = (int64_t)B;
            a.b_pos = (int32_t)pos_of(B);
            a.t = tv;
            const int o = cur ^ 1;
            a.d_key = dk[o]; a.d_pane = dp[o]; a.d_a0 = da0[o]; a.d_a1 = da1[o];
            a.st = d_st;
            if ((rc = clean_stale())) return rc;
            HIPCHECK(launch_merge_deferred(a, stream));
            cur = o;
            if ((rc = refresh())) return rc;
            if ((rc = take_occ())) return rc;
            if (!(h_st->flags & GW_DF_TABLE_FULL)) return GW_OK;
            if ((rc = maybe_grow(0))) return rc;  // grow, then retry the leftovers
            if ((int64_t)h_st->n_deferred == 0) return GW_OK;
            return merge_deferred();
        }
        return GW_OK;
    }

    int ensure_refire(int64_t need) {
        if (need <= rf_cap) return GW_OK;
        const int64_t nc = std::max<int64_t>(need + need / 2, 1 << 16);
        const int64_t used = std::min(rf_bound, rf_cap);
        for (int c = 0; c < 5; ++c) {
            int64_t* nb;
            HIPCHECK(hipMalloc((void**)&nb, nc * 8));
            if (rf[c] && used) HIPCHECK(hipMemcpyAsync(nb, rf[c], used * 8, hipMemcpyDeviceToDevice, stream));
            if (rf[c]) {
                HIPCHECK(hipStreamSynchronize(stream));
                hipFree(rf[c]);
            }
            rf[c] = nb;
        }
        rf_cap = nc;
        return GW_OK;
    }

    int ensure_late(int64_t need) {
        if (need <= lo_cap) return GW_OK;
        int rc;
        if ((rc = refresh())) return rc;  // exact n_late_out before copying
        const int64_t used = (int64_t)h_st->n_late_out;
        const int64_t nc = std::max<int64_t>(need + need / 2, 1 << 16);
        for (int c = 0; c < 3; ++c) {
            int64_t* nb;
            HIPCHECK(hipMalloc((void**)&nb, nc * 8));
            if (lo_buf[c] && used) HIPCHECK(hipMemcpyAsync(nb, lo_buf[c], used * 8, hipMemcpyDeviceToDevice, stream));
            if (lo_buf[c]) {
                HIPCHECK(hipStreamSynchronize(stream));
                hipFree(lo_buf[c]);
            }
            lo_buf[c] = nb;
        }
        lo_cap = nc;
        return GW_OK;
    }

    // Window index bounds under allowed lateness (WindowOperator.cleanupTime :670-677,
    // isWindowLate :609-612): window k is late at watermark w when max timestamp + lateness
    // <= w (a cleanup time beyond Long.MAX_VALUE is Long.MAX_VALUE: late only at the last
    // watermark, never cleaned), and its state is cleared by the cleanup timer once
    // max timestamp + lateness <= w < Long.MAX_VALUE.
    i128 k_for_wm128(i128 w) const { return floor_div(w + 1 - (i128)size() - (i128)cfg.offset, (i128)slide()); }
    i128 late_k_at(int64_t w) const {  // first window that is not late
        if (cfg.allowed_lateness == 0) return fired_k;
        const i128 k = w == INT64_MAX ? k_for_wm(w) + 1 : k_for_wm128((i128)w - cfg.allowed_lateness) + 1;
        return std::min(k, fired_k);
    }
    i128 clean_k_at(int64_t w) const {  // first window whose state is not cleared
        if (cfg.allowed_lateness == 0) return k_for_wm(w) + 1;
        return k_for_wm128(std::min<i128>(w, (i128)INT64_MAX - 1) - cfg.allowed_lateness) + 1;
    }

    // The re-fire list of the watermark interval that ends now: rows for every late
    // record of a fired, not yet cleaned window (k_refire), then the records go into the
    // table like parked ones.
    int process_refire() {
        if (!rf_bound) return GW_OK;
        int rc;
        if ((rc = refresh())) return rc;
        const int64_t nrf = (int64_t)h_st->n_refire;
        rf_bound = 0;
        if (nrf > kSortMaxRecords)  // one watermark's late records beyond the grouping sort
            return fail(GW_E_UNSUPPORTED, "%lld late records of fired windows between two watermarks (limit %lld)",
                        (long long)nrf, (long long)kSortMaxRecords);
        if (nrf) {
            const int64_t span = seq_ctr - rf_seq_base;
            const int seq_bits = span < ((int64_t)1 << 32) ? 32 : 64;
            const int64_t kb = ((nrf * 8 + 255) / 256) * 256, vb = ((nrf * 4 + 255) / 256) * 256;
            const int64_t need = 2 * kb + 2 * vb + radix_sort_scratch_bytes(nrf);
            if (need > rf_sort_bytes) {
                if (rf_sort) { HIPCHECK(hipStreamSynchronize(stream)); hipFree(rf_sort); }
                HIPCHECK(hipMalloc(&rf_sort, need + need / 2));
                rf_sort_bytes = need + need / 2;
            }
            char* base = (char*)rf_sort;
            uint64_t* k0 = (uint64_t*)base;
            uint64_t* k1 = (uint64_t*)(base + kb);
            uint32_t* v0 = (uint32_t*)(base + 2 * kb);
            uint32_t* v1 = (uint32_t*)(base + 2 * kb + vb);
            void* scratch = base + 2 * kb + 2 * vb;
            // (key, arrival) order: stable sort by arrival, then by key
            int alt = 0;
            HIPCHECK(launch_refire_keys(0, rf[4], rf_seq_base, k0, v0, nrf, stream));
            HIPCHECK(radix_sort_pairs(k0, v0, k1, v1, nrf, seq_bits, scratch, stream, &alt));
            uint64_t* ka = alt ? k0 : k1;  // the free key buffer
            uint32_t* va = alt ? v1 : v0;  // the sorted payload
            uint32_t* vo = alt ? v0 : v1;
            HIPCHECK(launch_refire_keys(1, rf[0], 0, ka, va, nrf, stream));
            uint64_t* kother = alt ? k1 : k0;
            HIPCHECK(radix_sort_pairs(ka, va, kother, vo, nrf, 64, scratch, stream, &alt));
            const uint32_t* order = alt ? vo : va;
            const int64_t per_rec = (n + m - 1) / m;  // windows a pane belongs to
            if ((rc = ensure_output((int64_t)h_st->rows + nrf * per_rec))) return rc;
            RefireArgs r{};
            r.t = tv;
            r.ov = ov_view();
            r.n = nrf;
            r.order = order;
            r.rf_key = rf[0]; r.rf_pane = rf[1]; r.rf_a0 = rf[2]; r.rf_a1 = rf[3];
            r.b = (int64_t)B;
            r.b_pos = (int32_t)pos_of(B);
            r.purging = cfg.trigger == GW_PURGING_EVENT_TIME_TRIGGER;
            r.m = (int64_t)m;
            r.np = (int64_t)n;
            r.k_lo = (int64_t)late_k_at(wm);
            r.k_hi = (int64_t)(fired_k - 1);
            r.offset = cfg.offset;
            r.slide = slide();
            r.size = size();
            r.o_key = o_key; r.o_start = o_start; r.o_end = o_end; r.o_res = o_res;
            r.st = d_st;
            if ((rc = rows_reset_now())) return rc;
            HIPCHECK(launch_refire(r, stream));
            // the records join their panes (windows that fire later fold them)
            if ((rc = ensure_deferred((int64_t)h_st->n_deferred + nrf))) return rc;
            MergeArgs a{};
            a.i_key = rf[0]; a.i_pane = rf[1]; a.i_a0 = rf[2]; a.i_a1 = rf[3];
            a.n = nrf;
            a.b = (int64_t)B;
            a.b_pos = (int32_t)pos_of(B);
            a.t = tv;
            a.d_key = dk[cur]; a.d_pane = dp[cur]; a.d_a0 = da0[cur]; a.d_a1 = da1[cur];
            a.st = d_st;
            if ((rc = clean_stale())) return rc;
            HIPCHECK(launch_merge_deferred(a, stream));
            if ((rc = set_field(offsetof(DevStatus, n_refire), 0))) return rc;
            dirty = true;
            if ((rc = refresh())) return rc;
            if ((rc = take_occ())) return rc;
            if (h_st->flags & GW_DF_TABLE_FULL) {
                if ((rc = maybe_grow(0))) return rc;
                if ((rc = merge_deferred())) return rc;
            }
        }
        rf_seq_base = seq_ctr;
        return GW_OK;
    }

    // Clear the ring panes below pane `upto` (their windows are fired and cleaned).
    // Presence-mask aggregates retire a pane by clearing its presence bits only (the cells
    // keep stale values behind them: 8 B per slot and position less to write per fire); the
    // positions are remembered and cleaned before a kernel that adds into cells with device
    // atomics (clean_stale).  The region apply and every reader go by the bits.
    // Lazy retires for the sums only: MIN / MAX retire eagerly (the fire writes the identity).
    // The apply's substitution of the identity for clear presence bits (k_rgn_apply_nar<AGG,
    // true>) cost Q7's tumbling max 335 -> 540 us per flush for ~25 us of fire per window; the
    // headline's sum pays ~1% of its apply for ~10% of its fire (profiles/r6/q7/).
    void lazy_retire(FireArgs& f) {
        const bool lazy = tv.has_mask && (cfg.agg == GW_SUM_I64 || cfg.agg == GW_SUM_I32 || cfg.agg == GW_SUM_F64);
        f.lazy_retire = lazy ? 1 : 0;
        if (lazy) stale_pos |= f.rmask;
    }
    int clean_stale() {
        if (!stale_pos) return GW_OK;
        HIPCHECK(launch_clean_stale(tv, stale_pos, stream));
        stale_pos = 0;
        return GW_OK;
    }

    int retire_below(i128 upto) {
        uint64_t rmask = 0;
        for (i128 p = B; p < upto && p < B + R; ++p) rmask |= 1ull << pos_of(p);
        rmask &= occ;
        if (rmask) {
            FireArgs f{};
            f.t = tv;
            f.nwin = 0;
            f.rmask = rmask;
            f.st = d_st;
            lazy_retire(f);
            HIPCHECK(launch_fire(f, stream));
            occ &= ~rmask;
            dirty = true;
        }
        if (B < upto) B = upto;
        return GW_OK;
    }

    // Lowest pane with data in the ring (or INT128 max).
    i128 ring_min() const {
        if (!occ) return ((i128)1) << 100;
        for (int j = 0; j < R; ++j)
            if (occ & (1ull << pos_of(B + j))) return B + j;
        return ((i128)1) << 100;
    }

    int deferred_min(i128& out) {
        out = ((i128)1) << 100;
        const int64_t nd = (int64_t)h_st->n_deferred;
        if (!nd) return GW_OK;
        int rc;
        if ((rc = set_field(offsetof(DevStatus, def_min_pane), (unsigned long long)INT64_MAX))) return rc;
        HIPCHECK(launch_deferred_min(dp[cur], nd, d_st, stream));
        if ((rc = refresh())) return rc;
        out = (i128)h_st->def_min_pane;
        return GW_OK;
    }

    // Move the ring base to pane nb (nb <= every pane holding data).
    int rebase(i128 nb) {
        int rc;
        if (nb < B) {
            // evicted positions may hold panes whose records are still carried: apply them first
            if (carry_on && (rc = flush_buffer())) return rc;
            uint64_t emask = 0;
            EvictArgs e{};
            for (i128 p = std::max(nb + R, B); p < B + R; ++p) {
                const int pos = (int)pos_of(p);
                if (occ & (1ull << pos)) {
                    emask |= 1ull << pos;
                    e.pane_of_pos[pos] = (int64_t)p;
                }
            }
            if (emask) {
                if ((rc = ensure_deferred((int64_t)h_st->n_deferred + (int64_t)(popcount(emask)) *
                                                                       ((int64_t)h_st->used_slots + 1))))
                    return rc;
                e.t = tv;
                e.emask = emask;
                e.d_key = dk[cur]; e.d_pane = dp[cur]; e.d_a0 = da0[cur]; e.d_a1 = da1[cur];
                e.st = d_st;
                HIPCHECK(launch_evict(e, stream));
                occ &= ~emask;
                if ((rc = refresh())) return rc;
            }
        }
        B = nb;
        return GW_OK;
    }
    static int popcount(uint64_t x) { return __builtin_popcountll(x); }

    // The fire of windows [k_first, k_last], retiring the ring positions of panes [B, keep).
    int fire_args(i128 k_first, i128 k_last, i128 keep, FireArgs& f, i128& keep_out) {
        const int nwin = (int)(k_last - k_first + 1);
        f.t = tv;
        f.ov = ov_view();
        f.k0 = (int64_t)k_first;
        f.nwin = nwin;
        const i128 start0 = (i128)cfg.offset + k_first * (i128)slide();
        const i128 endl = (i128)cfg.offset + k_last * (i128)slide() + size();
        if (!fits64(start0) || !fits64(endl)) return fail(GW_E_RANGE, "window bounds overflow int64");
        f.start0 = (int64_t)start0;
        f.slide = slide();
        f.size = size();
        for (int w = 0; w < nwin; ++w) {
            uint64_t wm_ = 0;
            const i128 p0 = (k_first + w) * m;
            for (int j = 0; j < n; ++j) wm_ |= 1ull << pos_of(p0 + j);
            f.wmask[w] = wm_;
        }
        uint64_t rmask = 0;
        for (i128 p = B; p < keep && p < B + R; ++p) rmask |= 1ull << pos_of(p);
        f.rmask = rmask;
        f.st = d_st;
        keep_out = keep;
        return GW_OK;
    }
    int fire_launch(const FireArgs& f) {
        int rc;
        if ((rc = rows_reset_now())) return rc;
        if (timing) {
            auto ev = t_fire.get();
            HIPCHECK(launch_fire(f, stream, ev.first, ev.second));
            t_fire.pending.push_back(ev);
        } else {
            HIPCHECK(launch_fire(f, stream));
        }
        return GW_OK;
    }
    // Host bookkeeping of a fire that ran.
    void fired(const FireArgs& f, i128 k_last, i128 keep) {
        stats.fires++;
        if (recs_since_fire) recs_per_fire = recs_since_fire, recs_since_fire = 0;
        dirty = true;
        occ &= ~f.rmask;
        fired_k = k_last + 1;
        if (B < keep) B = keep;
    }

    // Fire every window k <= k_target (end-1 <= wm).
    int fire_until(i128 k_target, i128 c_target) {
        int rc;
        const bool lat = cfg.allowed_lateness > 0;
        // panes below both frontiers belong to fired windows that are cleaned now
        if (lat && (rc = retire_below(std::min(fired_k, c_target) * m))) return rc;
        while (fired_k <= k_target) {
            i128 dmin;
            if ((rc = deferred_min(dmin))) return rc;
            const i128 rmin = ring_min();
            // restored windows whose timer is pending fire even without new records
            const i128 omin = ov_n ? ov_pending_min() * (i128)m + (i128)n - 1 : ((i128)1) << 100;
            const i128 L = std::min(std::min(rmin, dmin), omin);
            const i128 NONE = ((i128)1) << 100;
            if (L >= NONE) { fired_k = k_target + 1; break; }
            i128 k_first = floor_div(L - n, m) + 1;
            if (k_first < fired_k) k_first = fired_k;
            if (k_first > k_target) { fired_k = k_target + 1; break; }
            // keep the retained panes of fired, not yet cleaned windows in the ring
            if ((rc = rebase(lat ? std::min(k_first * m, L) : k_first * m))) return rc;
            if ((int64_t)h_st->n_deferred) {
                if ((rc = merge_deferred())) return rc;
            }
            i128 k_last = floor_div(B + R - n, m);
            if (k_last > k_target) k_last = k_target;
            if (k_last < k_first) return fail(GW_E_STATE, "pane ring too short for the retained panes");
            FireArgs f{};
            i128 keep;
            if ((rc = fire_args(k_first, k_last, lat ? std::min(k_last + 1, c_target) * m : (k_last + 1) * m, f,
                                keep)))
                return rc;
            if ((rc = ensure_output((int64_t)h_st->rows + (int64_t)f.nwin * ((int64_t)h_st->used_slots + 1))))
                return rc;
            f.o_key = o_key; f.o_start = o_start; f.o_end = o_end; f.o_res = o_res;
            lazy_retire(f);
            if ((rc = fire_launch(f))) return rc;
            fired(f, k_last, keep);
            if ((rc = refresh())) return rc;
        }
        if (lat) return retire_below(c_target * m);
        if (B < fired_k * m) B = fired_k * m;
        return GW_OK;
    }

    int64_t size() const { return cfg.assigner == GW_TUMBLING ? cfg.size : cfg.size; }
    int64_t slide() const { return cfg.assigner == GW_TUMBLING ? cfg.size : cfg.slide; }

    // Windows k <= K are complete at watermark wm: offset + k*slide + size - 1 <= wm.
    i128 k_for_wm(int64_t w) const {
        return floor_div((i128)w + 1 - (i128)size() - (i128)cfg.offset, (i128)slide());
    }

    // Ingest arguments shared by every path: the lateness bound and the ring geometry
    // at the current watermark.
    int base_args(IngestArgs& a, int64_t nrec, const int64_t* key, const int64_t* ts, const int64_t* val) {
        // first non-late pane: the first window that is not late at the current watermark
        // (lateness 0: the first window not fired)
        const i128 late_k = late_k_at(wm);
        const i128 p_late = late_k * m;
        i128 t_late = (i128)cfg.offset + p_late * g;
        i128 pl = p_late;
        int exact = 1;
        if (t_late <= (i128)INT64_MIN) {  // nothing can be late yet
            pl = floor_div((i128)INT64_MIN - cfg.offset + g - 1, g);
            t_late = (i128)cfg.offset + pl * g;
            exact = 0;
        }
        if (t_late > (i128)INT64_MAX) return fail(GW_E_RANGE, "watermark beyond the last representable window");
        if (B < pl) B = pl;
        a = IngestArgs{};
        a.key = key; a.ts = ts; a.val = val; a.n = nrec;
        a.pk_w = pk_w; a.pk_from = pk_from; a.pk_g = pk_g;
        a.t_late = (int64_t)t_late;
        a.p_late = (int64_t)pl;
        a.delta = (uint64_t)(B - pl);
        a.div = div;
        a.b_pos = (int32_t)pos_of(B);
        a.late_exact = exact;
        a.t = tv;
        a.cls_J = (int32_t)cls_J; a.cls_j = (int32_t)cls_j; a.cls_slide = cls_slide; a.cls_off = cls_off;
        a.gap_w = g; a.gap_size = gap_size;
        {
            const i128 gl = (i128)wm - (i128)cfg.allowed_lateness;
            a.gap_late = gl < (i128)INT64_MIN ? INT64_MIN : (int64_t)gl;
        }
        a.d_key = dk[cur]; a.d_pane = dp[cur]; a.d_a0 = da0[cur]; a.d_a1 = da1[cur];
        a.st = d_st;
        // panes up to the last one of the last fired window re-fire (lateness > 0)
        if (late_out() && exact) {
            int rc;
            if (nrec && (rc = ensure_late(lo_bound + nrec))) return rc;
            a.lo_key = lo_buf[0]; a.lo_ts = lo_buf[1]; a.lo_val = lo_buf[2];
        }
        const i128 hi = (fired_k - 1) * m + n - 1;
        if (late_k < fired_k && hi >= pl) {
            a.q_refire = (uint64_t)(hi - pl + 1);
            a.seq0 = seq_ctr;
            int rc;
            if (nrec && (rc = ensure_refire(rf_bound + nrec))) return rc;
            a.rf_key = rf[0]; a.rf_pane = rf[1]; a.rf_a0 = rf[2]; a.rf_a1 = rf[3]; a.rf_seq = rf[4];
        }
        return GW_OK;
    }

    // Region arrays of the current table geometry.
    void region_args(IngestArgs& a) {
        // 128 pass-1 buckets keep ~32 records per bucket run of a 4096-record tile
        a.d1_bits = tv.rb1;
        a.two_pass = tv.nsub > 1;
        a.p1_key = e_col[3]; a.p1_a0 = e_col[4]; a.p1_a1 = e_col[5]; a.p1_pos = e_pos[1];
        a.e_key = eset_key(eset); a.e_a0 = e_col[1]; a.e_a1 = e_col[2]; a.e_pos = e_pos[0];
        a.p1_row = p1_row;
        a.p2_desc = p2_desc;
        a.p2_off = p2_off;
        a.stale = stale_pos != 0;
        a.p2_roff = p2_roff;
        a.rbeg = eset_rbeg(eset);
        a.bk_off = a.rbeg + kPartBuckets + 1;
        a.r_row = eset_row(eset);
        a.r_base = eset_base(eset);
        a.apply_mask = ~0ull;
        a.batch_occ = d_tmp + 1;
        a.fmt = buf_fmt;
        nar_mode(a);
    }

    // Narrow records of two-pass tables: P2 groups each round by (super-region, ring position)
    // and k_rgn_apply_nar applies a super-region one position after another (nar2).  Fixed per
    // flush window: the format and the table geometry do not change while segments wait.
    void nar_mode(IngestArgs& a) const {
        // narrow records of two-pass tables: k_rgn_apply_nar over super-regions of F regions
        // (GW_NAR_F = 1, 2 or 4, default 2; GW_NAR2=0 keeps k_rgn_apply), while P2's (super-region,
        // ring position) buckets fit a descriptor row
        static const int nar_f = [] {
            const char* e = getenv("GW_NAR_F");
            const int f = e ? atoi(e) : 2;
            return f >= 4 ? 2 : f >= 2 ? 1 : 0;
        }();
        static const bool nar2_off = [] { const char* e = getenv("GW_NAR2"); return e && atoi(e) == 0; }();
        a.nar2 = 0;
        a.sr_bits = 0;
        if (buf_fmt == 2 && a.two_pass && !nar2_off && tv.ring <= 8) {
            int sr = nar_f;
            while ((tv.nsub >> sr) > 32) ++sr;  // (super-region << 3 | position) < kPartBuckets
            if (sr <= 2 && tv.nsub % (1 << sr) == 0) {
                a.nar2 = 1;
                a.sr_bits = sr;
            }
        }
    }

    // Compact region records (gw_pane.hip cmp_pack): integer aggregates whose ring
    // positions fit below the pass-1 bucket bits (R <= 2^(d1-1)).
    bool compact_ok(int d1_bits) const {
        const int agg = cfg.agg;
        const bool int_agg = agg == GW_COUNT || agg == GW_SUM_I64 || agg == GW_SUM_I32 || agg == GW_MIN_I64 ||
                             agg == GW_MAX_I64 || agg == GW_AVG_I64;
        static const bool env_off = getenv("GW_NO_COMPACT") != nullptr;
        // gapped panes (size < slide) use the wide pass 1, the one instantiated with the gap test
        return int_agg && !cmp_off && !env_off && !gap_size && d1_bits >= 2 && (int64_t)tv.ring <= ((int64_t)1 << (d1_bits - 1));
    }
    // Narrow records (32-bit keys, 28-bit values, ring positions < 8) for integer aggregates
    // whose windows have not overflowed them yet (GW_NO_NARROW turns them off).  They keep
    // the ring position beside the key, so unlike compact records they need no spare
    // pass-1 bucket bits (small single-pass tables under allowed lateness take them too).
    int region_fmt(int d1_bits) const {
        const int agg = cfg.agg;
        const bool int_agg = agg == GW_COUNT || agg == GW_SUM_I64 || agg == GW_SUM_I32 || agg == GW_MIN_I64 ||
                             agg == GW_MAX_I64 || agg == GW_AVG_I64;
        static const bool nar_env_off = getenv("GW_NO_NARROW") != nullptr;
        static const bool cmp_env_off = getenv("GW_NO_COMPACT") != nullptr;
        if (int_agg && !gap_size && !cmp_env_off && !nar_off && !nar_env_off && !(cfg.flags & GW_FLAG_NO_NARROW) &&
            tv.ring <= 8)
            return 2;
        return compact_ok(d1_bits) ? 1 : 0;
    }

    // P2 + apply over every waiting segment (one fire's worth of batches).  Runs before
    // any fire, rehash, merge or non-region ingest, so the table is exact whenever it is
    // read.
    // apply_mask (a fire, nar2 only): ring positions that must be applied now; the others may
    // stay in this flush's P2 output until the next flush (carry).  Every other caller applies
    // everything, carried positions included.
    // A flush is its launches (flush_launch: false when there is nothing to apply) and what the
    // host does once the status after them is exact (flush_post, after a refresh).
    struct PendingFlush {
        IngestArgs a;
        int64_t window_recs = 0;
    };
    int flush_buffer(uint64_t apply_mask = ~0ull) {
        PendingFlush pf;
        bool launched = false;
        int rc;
        if ((rc = flush_launch(apply_mask, pf, launched)) || !launched) return rc;
        if ((rc = refresh())) return rc;
        return flush_post(pf);
    }
    int flush_launch(uint64_t apply_mask, PendingFlush& pf, bool& launched) {
        launched = false;
        if (!nseg && !carry_on) return GW_OK;
        int rc;
        IngestArgs& a = pf.a;
        if ((rc = base_args(a, 0, nullptr, nullptr, nullptr))) return rc;
        region_args(a);
        if (carry_on && !a.nar2) return fail(GW_E_STATE, "internal: carried records without a nar2 flush");
        a.ntiles = buf_tiles;
        a.p2_group = region_group(a.d1_bits);
        a.ngroups = (buf_tiles + a.p2_group - 1) / a.p2_group;
        a.ring_fresh = buf_fresh;
        a.cur_empty = nseg == 0;
        if (carry_on) {
            const int c = eset ^ 1;
            a.c_mask = carry_mask;
            a.c_key = eset_key(c);
            a.c_r_row = eset_row(c);
            a.c_r_base = eset_base(c);
            a.c_rbeg = eset_rbeg(c);
        }
        // carry only what a fire leaves behind, on the plain path (no lateness, no restored
        // windows); at most one flush deep
        uint64_t carry_next = 0;
        static const bool carry_off = [] { const char* e = getenv("GW_NAR_CARRY"); return e && atoi(e) == 0; }();
        if (a.nar2 && nseg && apply_mask != ~0ull && cfg.allowed_lateness == 0 && ov_n == 0 && !carry_off) {
            const uint64_t ring = R >= 64 ? ~0ull : ((1ull << R) - 1);
            carry_next = ring & ~apply_mask;
            a.apply_mask = apply_mask;
            // the next P2 writes the other set; the one carried so far is applied by this flush
            if (carry_next && (rc = ensure_eset2())) return rc;
        }
        const int64_t window_recs = buf_recs;
        nseg = 0;  // before any launch: the TABLE_FULL handling below may grow the table
        buf_tiles = 0;
        buf_recs = 0;
        carry_on = false;
        if (carry_next) {
            carry_on = true;
            carry_mask = carry_next;
            eset ^= 1;
        }
        if (timing) {
            auto ev = t_apply.get();
            HIPCHECK(launch_region_flush(a, stream, ev.first, ev.second));
            t_apply.pending.push_back(ev);
        } else {
            HIPCHECK(launch_region_flush(a, stream));
        }
        // the next window's pass-1 occupancy word, zeroed while the device is still busy (behind
        // the apply that read it) instead of on the host's critical path at its first pass 1
        HIPCHECK(hipMemsetAsync(d_tmp + 1, 0, 8, stream));
        occ_zeroed = true;
        stats.applies++;
        dirty = true;
        launched = true;
        pf.window_recs = window_recs;
        return GW_OK;
    }
    int flush_post(PendingFlush& pf) {
        int rc;
        IngestArgs& a = pf.a;
        if (h_st->wide_vals) {  // records beyond the window's format went the deferred way: keep it rare
            if (h_st->wide_vals * 64 > (unsigned long long)pf.window_recs) {
                if (a.fmt == 2) nar_off = true;
                else cmp_off = true;
            }
            if ((rc = set_field(offsetof(DevStatus, wide_vals), 0))) return rc;
        }
        if (h_st->spills) {  // full regions / a third ring position left records: park them
            if ((rc = ensure_deferred((int64_t)h_st->n_deferred + (int64_t)h_st->spills))) return rc;
            if ((rc = set_field(offsetof(DevStatus, spills), 0))) return rc;
            HIPCHECK(launch_region_collect(a, stream));
            dirty = true;
            if ((rc = refresh())) return rc;
            if (!(h_st->flags & GW_DF_TABLE_FULL) && (rc = merge_deferred())) return rc;
        }
        if (h_st->flags & GW_DF_TABLE_FULL) {
            if ((rc = maybe_grow(0))) return rc;
            if ((rc = merge_deferred())) return rc;
        }
        return GW_OK;
    }

    // The packed words of the current batch unpacked behind its other records, in pk_stage;
    // key / ts / val then point there and the batch has no words any more.
    int pk_materialize(int64_t nrec, const int64_t*& key, const int64_t*& ts, const int64_t*& val) {
        if (nrec > pk_stage_cap) {
            HIPCHECK(hipStreamSynchronize(stream));
            hipFree(pk_stage);
            pk_stage = nullptr;
            const int64_t c = std::max<int64_t>(nrec + nrec / 4, 1 << 16);
            HIPCHECK(hipMalloc((void**)&pk_stage, (size_t)c * 3 * 8));
            pk_stage_cap = c;
        }
        int64_t* k = pk_stage;
        int64_t* t = k + pk_stage_cap;
        int64_t* v = val ? t + pk_stage_cap : nullptr;
        if (pk_from > 0) {
            HIPCHECK(hipMemcpyAsync(k, key, (size_t)pk_from * 8, hipMemcpyDeviceToDevice, stream));
            HIPCHECK(hipMemcpyAsync(t, ts, (size_t)pk_from * 8, hipMemcpyDeviceToDevice, stream));
            if (v) HIPCHECK(hipMemcpyAsync(v, val, (size_t)pk_from * 8, hipMemcpyDeviceToDevice, stream));
        }
        HIPCHECK(launch_unpack(nrec - pk_from, pk_w, pk_g, k + pk_from, t + pk_from, v ? v + pk_from : nullptr, stream));
        key = k;
        ts = t;
        val = v;
        pk_w = nullptr;
        pk_from = 0;
        return GW_OK;
    }

    int ingest_pane(int64_t nrec, const int64_t* key, const int64_t* ts, const int64_t* val) {
        int rc;
        if ((rc = ov_finalize())) return rc;
        hp.lap(6);
        if (dirty && (rc = refresh())) return rc;  // a lagging (lazy) status is fine here
        hp.lap(7);
        if ((rc = maybe_grow(nrec))) return rc;
        hp.lap(8);
        // room for every deferred entry the launches since the last exact status may have
        // written; when that bound outgrows the list, learn the exact count first (one sync)
        // rather than growing it by the bound (a reallocation: a sync and a copy) -- the bound
        // keeps growing while host writes leave the published status slots stale
        if (lazy_recs > 0 && (int64_t)h_st->n_deferred + lazy_recs + nrec > def_cap) {
            if (hp.on)
                fprintf(stderr, "[gw host] deferred bound: n_deferred %lld lazy %lld nrec %lld cap %lld\n",
                        (long long)h_st->n_deferred, (long long)lazy_recs, (long long)nrec, (long long)def_cap);
            if ((rc = refresh())) return rc;
            // and grow the list to n_deferred + (kAsync + 1) batches (this sync has happened
            // anyway): the steady state leaves kAsync batches' launches unaccounted, and a list
            // sized for fewer synced here on every batch.  Measured (profiles/r5/defgrow/): Q5
            // at 1M-record batches 11.5 G against 10.4 G (after a 15-batch warmup: the one
            // reallocation, ~1.5 ms, lands in the first region-path batch), at 10M-record
            // batches 50.5 G against 49.0 G.  GW_DEF_GROW=0: the round-4 policy.
            static const int grow = getenv("GW_DEF_GROW") ? atoi(getenv("GW_DEF_GROW")) : kAsync + 1;
            if (grow && (rc = ensure_deferred((int64_t)h_st->n_deferred + grow * nrec))) return rc;
        }
        if ((rc = ensure_deferred((int64_t)h_st->n_deferred + lazy_recs + nrec))) return rc;
        hp.lap(9);
        IngestArgs a;
        if ((rc = base_args(a, nrec, key, ts, val))) return rc;
        hp.lap(10);
        // path: LDS pre-aggregation when the batch repeats few keys many times; region
        // bucketing when the batch is large against the table (its streaming passes cost
        // ~48 B per slot, the direct path ~300 B of scattered traffic per record);
        // otherwise direct atomics.
        int path = 0;
        const int64_t est = h_st->used_slots ? (int64_t)h_st->used_slots : cfg.capacity_hint;
        if (cfg.flags & GW_FLAG_FORCE_LDS_PREAGG) path = 1;
        else if (!(cfg.flags & GW_FLAG_NO_LDS_PREAGG) && est > 0 && nrec >= 8 * est) path = 1;
        if (path == 0 && tv.nreg <= kRgnMaxRegions && !(cfg.flags & GW_FLAG_NO_REGION)) {
            // large against the table: the batch itself, or (two-pass tables buffer until the
            // fire) the last fire cycle's records
            const bool cycle = tv.nsub > 1 && !(cfg.flags & GW_FLAG_NO_BUFFER) &&  // two-pass
                               recs_per_fire * 8 >= tv.cap;
            const bool big = nrec >= region_min_batch && (nrec * 8 >= tv.cap || cycle);
            if (big || (cfg.flags & GW_FLAG_FORCE_REGION)) path = 2;
        }
        if (path == 1) stats.preagg_batches++;
        if (pk_w && (path != 2 || a.lo_key)) {  // only the region P1 decodes packed words
            if ((rc = pk_materialize(nrec, key, ts, val))) return rc;
            if ((rc = base_args(a, nrec, key, ts, val))) return rc;
        }
        if (path != 2 && (nseg || carry_on)) {  // the other paths write the table directly: apply first
            if ((rc = flush_buffer())) return rc;
            if ((rc = base_args(a, nrec, key, ts, val))) return rc;  // the table may have grown
        }
        hp.lap(11);
        if (path == 2) {
            region_args(a);
            // Two-pass tables buffer P1 segments across watermarks (P2 + apply once per
            // fire); single-pass tables apply every batch.
            const bool buffered = a.two_pass && !(cfg.flags & GW_FLAG_NO_BUFFER);
            const int64_t tiles = (nrec + kPartTile - 1) / kPartTile;
            if (nseg && buf_tiles + tiles > buf_cap) {
                if ((rc = flush_buffer())) return rc;
                if ((rc = base_args(a, nrec, key, ts, val))) return rc;
            }
            const int64_t want =
                buffered ? std::min(std::max<int64_t>(buf_limit / kPartTile, 1), std::max<int64_t>(16 * tiles, 256))
                         : tiles;
            if ((rc = ensure_region(buf_tiles + tiles, want))) return rc;
            region_args(a);
            a.tile0 = buf_tiles;
            hp.lap(12);
            if (nseg == 0) {
                const int fmt = region_fmt(a.d1_bits);
                if (carry_on && fmt != buf_fmt) {  // carried records keep their window's format: apply them
                    if ((rc = flush_buffer())) return rc;
                    if ((rc = base_args(a, nrec, key, ts, val))) return rc;
                    region_args(a);
                    a.tile0 = buf_tiles;
                }
                if (!occ_zeroed) HIPCHECK(hipMemsetAsync(d_tmp + 1, 0, 8, stream));
                occ_zeroed = false;
                buf_fresh = ~occ;
                buf_fmt = fmt;
            }
            a.fmt = buf_fmt;
            nar_mode(a);
            stats.region_format = buf_fmt;
            if (buffered) arm_status(a);
            hp.lap(13);
            if (timing && (timing_ctr++ % timing_every) == 0) {  // every timing_every-th batch
                auto ev = t_ingest.get();
                HIPCHECK(launch_region_p1(a, stream, ev.first, ev.second));
                t_ingest.pending.push_back(ev);
            } else {
                HIPCHECK(launch_region_p1(a, stream));
            }
            nseg++;
            buf_tiles += tiles;
            buf_recs += nrec;
            if (!buffered && (rc = flush_buffer())) return rc;
        } else if ((rc = clean_stale())) {
            return rc;
        } else if (timing) {
            auto ev = t_ingest.get();
            HIPCHECK(hipEventRecord(ev.first, stream));
            HIPCHECK(launch_ingest(a, path, ingest_unroll, stream));
            HIPCHECK(hipEventRecord(ev.second, stream));
            t_ingest.pending.push_back(ev);
        } else {
            HIPCHECK(launch_ingest(a, path, ingest_unroll, stream));
        }
        stats.events_in += nrec;
        stats.batches++;
        seq_ctr += nrec;
        recs_since_fire += nrec;
        if (a.lo_key) lo_bound += nrec;
        if (a.q_refire) rf_bound += nrec;
        if (path == 2 && nseg) {  // buffered P1: no host sync (it writes no table cell)
            if ((rc = lazy_status(nrec))) return rc;
            if (occ || !h_st->n_deferred) return GW_OK;
        }
        dirty = true;
        if ((rc = refresh())) return rc;  // the host sync of an unbuffered ingest call
        if (h_st->flags & GW_DF_TABLE_FULL) {
            if ((rc = maybe_grow(0))) return rc;
            if ((rc = merge_deferred())) return rc;
        }
        // An empty ring with parked records: jump the ring to the data (the buffer holds
        // no in-ring record then; apply it before the ring moves all the same).
        if (!occ && h_st->n_deferred && (nseg || carry_on) && (rc = flush_buffer())) return rc;
        if (!occ && h_st->n_deferred) {
            i128 dmin;
            if ((rc = deferred_min(dmin))) return rc;
            const i128 lo = late_k_at(wm) * m;
            B = rf_bound ? lo : std::max(lo, dmin);  // pending re-fire records sit at >= lo
            if ((rc = merge_deferred())) return rc;
        }
        return GW_OK;
    }

    // ---------------------------------------------------------------- key checks
    // Synchronous: only callers that pass a key_hash column or set GW_FLAG_CHECK_KEY_GROUPS
    // pay for it (the Java operator passes no hash for Long keys).
    int check_keys(int64_t nrec, const int64_t* d_key, const int32_t* d_hash) {
        const bool range = (cfg.flags & GW_FLAG_CHECK_KEY_GROUPS) != 0;
        if (nrec == 0 || (!d_hash && !range)) return GW_OK;
        if (!d_chk) HIPCHECK(hipMalloc((void**)&d_chk, 32));
        const unsigned long long init[4] = {0ull, ~0ull, 0ull, 0ull};
        HIPCHECK(hipMemcpyAsync(d_chk, init, 32, hipMemcpyHostToDevice, stream));
        const int32_t mp = cfg.max_parallelism, p = cfg.parallelism, ix = cfg.operator_index;
        const int32_t lo = (ix * mp + p - 1) / p, hi = ((ix + 1) * mp - 1) / p;  // KeyGroupRangeAssignment :93-106
        HIPCHECK(launch_check_keys(nrec, d_key, d_hash, mp, lo, hi, range ? 1 : 0, d_chk, stream));
        if (d_hash) {  // remember each key's hash: snapshots file its state under that key group
            int rc = khm_reserve(nrec);
            if (rc) return rc;
            HIPCHECK(launch_khmap_insert(khm, nrec, d_key, d_hash, 0, d_chk + 2, stream));
            HIPCHECK(launch_khmap_insert(khm, nrec, d_key, d_hash, 1, d_chk + 2, stream));
        }
        unsigned long long out[4];
        HIPCHECK(hipMemcpyAsync(out, d_chk, 32, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        khm_used += (int64_t)out[2];
        if (out[3]) {
            failed = true;
            return fail(GW_E_INVALID, "a key arrived with two different key hashes (hashCode is not deterministic)");
        }
        if (out[0]) foreign_hash = true;
        if (out[1] != ~0ull) {
            failed = true;
            return fail(GW_E_INVALID,
                        "Key group %d is not in KeyGroupRange{startKeyGroup=%d, endKeyGroup=%d}. Unless you're "
                        "directly using low level state access APIs, this is most likely caused by "
                        "non-deterministic shuffle key (hashCode and equals implementation).",
                        (int)(out[1] - 1), lo, hi);
        }
        return GW_OK;
    }

    // ------------------------------------------------- key -> Java hashCode (KeyHashMap)
    KeyHashMap khm{};
    int64_t khm_used = 0;  // keys in khm
    void khm_free() {
        if (khm.key) hipFree(khm.key);
        if (khm.hash) hipFree(khm.hash);
        khm = KeyHashMap{};
        khm_used = 0;
    }
    // Room for `more` new keys at load <= 0.5 (grows by rehashing).
    int khm_reserve(int64_t more) {
        if (khm.cap && 2 * (khm_used + more) <= khm.cap) return GW_OK;
        int64_t cap = khm.cap ? khm.cap : 1 << 12;
        while (2 * (khm_used + more) > cap) cap *= 2;
        KeyHashMap n;
        n.cap = cap;
        if (hipMalloc((void**)&n.key, (size_t)(cap + 1) * 8) != hipSuccess ||
            hipMalloc((void**)&n.hash, (size_t)(cap + 1) * 4) != hipSuccess) {
            if (n.key) hipFree(n.key);
            return fail(GW_E_OOM, "key-hash map: out of device memory");
        }
        HIPCHECK(launch_fill64(n.key, cap, kEmptyKey, stream));
        HIPCHECK(hipMemsetAsync(n.key + cap, 0, 8, stream));
        HIPCHECK(hipMemsetAsync(n.hash + cap, 0, 4, stream));
        if (khm.cap) HIPCHECK(launch_khmap_rehash(khm, n, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        const int64_t used = khm_used;
        khm_free();
        khm = n;
        khm_used = used;
        return GW_OK;
    }
    // Host copy of the map, sorted by key, for key groups at snapshot time.
    struct KhmHost {
        std::vector<std::pair<int64_t, int32_t>> kv;
        bool has_min = false;
        int32_t min_hash = 0;
        bool on() const { return has_min || !kv.empty(); }
        int32_t hash(int64_t key) const {
            if (key == kEmptyKey) return has_min ? min_hash : java_long_hash(key);
            auto it = std::lower_bound(kv.begin(), kv.end(), std::make_pair(key, INT32_MIN));
            return it != kv.end() && it->first == key ? it->second : java_long_hash(key);
        }
    };
    int khm_host(KhmHost& out) {
        out = KhmHost{};
        if (!khm_used) return GW_OK;
        std::vector<int64_t> k((size_t)khm.cap + 1);
        std::vector<int32_t> h((size_t)khm.cap + 1);
        HIPCHECK(hipStreamSynchronize(stream));
        HIPCHECK(hipMemcpy(k.data(), khm.key, k.size() * 8, hipMemcpyDeviceToHost));
        HIPCHECK(hipMemcpy(h.data(), khm.hash, h.size() * 4, hipMemcpyDeviceToHost));
        out.kv.reserve((size_t)khm_used);
        for (int64_t i = 0; i < khm.cap; ++i)
            if (k[i] != kEmptyKey) out.kv.push_back({k[i], h[i]});
        std::sort(out.kv.begin(), out.kv.end());
        out.has_min = k[khm.cap] != 0;
        out.min_hash = h[khm.cap];
        return GW_OK;
    }
    // (key, hash) pairs of a restored blob into the map.
    int khm_insert_host(const std::vector<int64_t>& keys, const std::vector<int32_t>& hashes) {
        const int64_t n = (int64_t)keys.size();
        if (!n) return GW_OK;
        int rc = khm_reserve(n);
        if (rc) return rc;
        int64_t* dk_ = nullptr;
        int32_t* dh_ = nullptr;
        if (!d_chk) HIPCHECK(hipMalloc((void**)&d_chk, 32));
        HIPCHECK(hipMalloc((void**)&dk_, (size_t)n * 8));
        HIPCHECK(hipMalloc((void**)&dh_, (size_t)n * 4));
        HIPCHECK(hipMemcpy(dk_, keys.data(), (size_t)n * 8, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dh_, hashes.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        const unsigned long long init[4] = {0ull, ~0ull, 0ull, 0ull};
        HIPCHECK(hipMemcpyAsync(d_chk, init, 32, hipMemcpyHostToDevice, stream));
        HIPCHECK(launch_khmap_insert(khm, n, dk_, dh_, 0, d_chk + 2, stream));
        HIPCHECK(launch_khmap_insert(khm, n, dk_, dh_, 1, d_chk + 2, stream));
        unsigned long long out[4];
        HIPCHECK(hipMemcpyAsync(out, d_chk, 32, hipMemcpyDeviceToHost, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        hipFree(dk_);
        hipFree(dh_);
        khm_used += (int64_t)out[2];
        if (out[3]) return fail(GW_E_INVALID, "snapshot: a key with two different key hashes");
        return GW_OK;
    }

    // A restored blob's (key, hash) pairs, checked on the host before anything changes: one
    // hash per key within the blob and the same hash as the map already holds for that key.
    int khm_check_host(const std::vector<int64_t>& keys, const std::vector<int32_t>& hashes) {
        if (keys.empty()) return GW_OK;
        std::vector<std::pair<int64_t, int32_t>> kv(keys.size());
        for (size_t i = 0; i < keys.size(); ++i) kv[i] = {keys[i], hashes[i]};
        std::sort(kv.begin(), kv.end());
        for (size_t i = 1; i < kv.size(); ++i)
            if (kv[i].first == kv[i - 1].first && kv[i].second != kv[i - 1].second)
                return fail(GW_E_INVALID, "snapshot: a key with two different key hashes");
        if (!khm_used) return GW_OK;
        KhmHost kh;
        int rc = khm_host(kh);
        if (rc) return rc;
        for (const auto& e : kv) {
            bool known = false;
            int32_t h0 = 0;
            if (e.first == kEmptyKey) {
                known = kh.has_min;
                h0 = kh.min_hash;
            } else {
                auto it = std::lower_bound(kh.kv.begin(), kh.kv.end(), std::make_pair(e.first, INT32_MIN));
                if (it != kh.kv.end() && it->first == e.first) { known = true; h0 = it->second; }
            }
            if (known && h0 != e.second) return fail(GW_E_INVALID, "snapshot: a key with two different key hashes");
        }
        return GW_OK;
    }

    // ---------------------------------------------------------------- snapshot
    // Blob (little-endian): SnapHeader, int64 kg_offsets[kg_hi - kg_lo + 2], then the entries
    // of each key group.  Versions: 2 session windows, 3 count windows (fixed-size entries of
    // `reserved` int64 words, offsets in entries), 4 tumbling / sliding windows (the heap
    // backend's per-key-group byte layout, offsets in bytes; see snapshot_heap).
    // flags: kSnapKeyHashes -- the keys came with a key_hash column (String, Integer, ...
    // keys as caller ids): each state entry carries the key's Java hashCode after the key
    // (version 4: be32 after the be64 key; versions 2 / 3: one more int64 word at the end).
    struct SnapHeader {
        char magic[4];
        uint32_t version;
        int32_t agg, assigner;
        int64_t size, slide, offset, gap, flags;
        int32_t max_parallelism, kg_lo, kg_hi, reserved;
        int64_t fired_lo, fired_hi;
        int64_t entries;  // entries (versions 2, 3) / payload bytes (version 4)
    };

    // -------------------------------------------- restored window state (the overlay)
    // A heap-layout blob holds the reference's state per (key, window) and its timers.
    // Windows overlap (sliding), so a window's accumulator cannot be split back into panes:
    // it stays a window-level entry (gw_kernels.h Overlay) that k_fire / k_refire fold
    // into the window's row together with the panes of the records that arrive after the
    // restore.  The watermark restarts at Long.MIN_VALUE as in the reference
    // (InternalTimerServiceImpl.java:72): nothing has fired, nothing is late.
    struct OvEntry {
        int64_t key, k, a0, a1;
        uint32_t flags;
    };
    std::vector<OvEntry> ov_pending;  // restored, not yet on the device
    int64_t* d_ov = nullptr;          // key | k | a0 | a1, ov_n each
    uint32_t* d_ov_flags = nullptr;
    int32_t* d_ov_head = nullptr;     // [tv.cap + 1]
    int64_t ov_n = 0, ov_nkeys = 0;
    i128 ov_max_k = 0;
    std::vector<int64_t> ov_timer_ks;  // sorted window indices with a pending timer

    Overlay ov_view() const {
        Overlay o{};
        if (!ov_n) return o;
        o.head = d_ov_head;
        o.key = d_ov; o.k = d_ov + ov_n; o.a0 = d_ov + 2 * ov_n; o.a1 = d_ov + 3 * ov_n;
        o.flags = d_ov_flags;
        o.n = ov_n;
        o.purge = cfg.allowed_lateness == 0 || cfg.trigger == GW_PURGING_EVENT_TIME_TRIGGER;
        return o;
    }
    void ov_free() {
        if (d_ov) hipFree(d_ov);
        if (d_ov_flags) hipFree(d_ov_flags);
        if (d_ov_head) hipFree(d_ov_head);
        d_ov = nullptr; d_ov_flags = nullptr; d_ov_head = nullptr;
        ov_n = ov_nkeys = 0;
        ov_timer_ks.clear();
    }
    // Slots of the overlay keys in the current table (after the restore and every rehash).
    int ov_attach() {
        if (!ov_n) return GW_OK;
        if (d_ov_head) HIPCHECK(hipFree(d_ov_head));
        HIPCHECK(hipMalloc((void**)&d_ov_head, (size_t)(tv.cap + 1) * 4));
        HIPCHECK(hipMemsetAsync(d_ov_head, 0xff, (size_t)(tv.cap + 1) * 4, stream));
        HIPCHECK(launch_overlay_attach(tv, ov_view(), d_ov_head, d_st, stream));
        dirty = true;
        int rc;
        if ((rc = refresh())) return rc;
        if (h_st->flags & GW_DF_TABLE_FULL) return fail(GW_E_OOM, "state table full attaching restored state");
        return GW_OK;
    }
    // Move the restored entries to the device (first call after the restores).
    int ov_finalize() {
        if (ov_pending.empty()) return GW_OK;
        auto& v = ov_pending;
        std::sort(v.begin(), v.end(), [](const OvEntry& x, const OvEntry& y) {
            return x.key != y.key ? x.key < y.key : x.k < y.k;
        });
        size_t w = 0;  // one entry per (key, window): merge repeats (the same key group twice)
        for (size_t i = 0; i < v.size(); ++i) {
            if (w && v[w - 1].key == v[i].key && v[w - 1].k == v[i].k) {
                fold_cell(cfg.agg, v[w - 1].a0, v[w - 1].a1, v[i].a0, v[i].a1);
                v[w - 1].flags |= v[i].flags;
            } else {
                v[w++] = v[i];
            }
        }
        v.resize(w);
        const int64_t n = (int64_t)w;
        ov_free();
        std::vector<int64_t> cols((size_t)n * 4);
        std::vector<uint32_t> fl((size_t)n);
        ov_nkeys = 0;
        ov_max_k = v.empty() ? 0 : v[0].k;
        for (int64_t i = 0; i < n; ++i) {
            cols[i] = v[i].key; cols[n + i] = v[i].k; cols[2 * n + i] = v[i].a0; cols[3 * n + i] = v[i].a1;
            fl[i] = v[i].flags;
            if (v[i].flags & kOvTimer) ov_timer_ks.push_back(v[i].k);
            if (i == 0 || v[i].key != v[i - 1].key) ov_nkeys++;
            if (v[i].k > ov_max_k) ov_max_k = v[i].k;
        }
        std::sort(ov_timer_ks.begin(), ov_timer_ks.end());
        ov_timer_ks.erase(std::unique(ov_timer_ks.begin(), ov_timer_ks.end()), ov_timer_ks.end());
        ov_pending.clear();
        if (!n) return GW_OK;
        HIPCHECK(hipMalloc((void**)&d_ov, (size_t)n * 32));
        HIPCHECK(hipMalloc((void**)&d_ov_flags, (size_t)n * 4));
        HIPCHECK(hipMemcpy(d_ov, cols.data(), (size_t)n * 32, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(d_ov_flags, fl.data(), (size_t)n * 4, hipMemcpyHostToDevice));
        ov_n = n;
        int rc;
        // room for the restored keys before they get slots
        if ((double)(h_st->used_slots + ov_nkeys) > 0.7 * (double)tv.cap) {
            int64_t want = tv.cap;
            while ((double)(h_st->used_slots + ov_nkeys) > 0.5 * (double)want) want *= 2;
            if ((rc = rehash(want))) return rc;  // attaches
            return GW_OK;
        }
        return ov_attach();
    }
    // Smallest window index >= fired_k whose restored timer is pending (or "none").
    i128 ov_pending_min() const {
        auto it = std::lower_bound(ov_timer_ks.begin(), ov_timer_ks.end(), (int64_t)std::max<i128>(fired_k, INT64_MIN));
        return it == ov_timer_ks.end() ? ((i128)1) << 100 : (i128)*it;
    }
    // Every restored window is fired and cleaned: drop the overlay.
    void ov_maybe_release(int64_t w) {
        if (ov_n && clean_k_at(w) > ov_max_k && fired_k > ov_max_k) ov_free();
    }

    // Accumulator <-> cell words (the serializer's value, gw_common.h cells).
    void acc_to_be(std::vector<uint8_t>& o, int64_t a0, int64_t a1) const {
        switch (cfg.agg) {
        case GW_SUM_I32: be32(o, (int32_t)(uint32_t)(uint64_t)a0); break;
        case GW_MIN_F64: case GW_MAX_F64: be64(o, f64_from_order_key(a0)); break;
        case GW_AVG_I64: case GW_AVG_F64: be64(o, a0); be64(o, a1); break;
        default: be64(o, a0); break;
        }
    }
    int acc_bytes() const {
        return cfg.agg == GW_SUM_I32 ? 4 : (cfg.agg == GW_AVG_I64 || cfg.agg == GW_AVG_F64) ? 16 : 8;
    }
    void acc_from_be(const uint8_t* p, int64_t& a0, int64_t& a1) const {
        a1 = 0;
        switch (cfg.agg) {
        case GW_SUM_I32: a0 = (int64_t)rd32(p); break;
        case GW_MIN_F64: case GW_MAX_F64: a0 = f64_order_key(rd64(p)); break;
        case GW_AVG_I64: case GW_AVG_F64: a0 = rd64(p); a1 = rd64(p + 8); break;
        default: a0 = rd64(p); break;
        }
    }
    static void be64(std::vector<uint8_t>& o, int64_t v) {
        for (int i = 0; i < 8; ++i) o.push_back((uint8_t)((uint64_t)v >> (56 - 8 * i)));
    }
    static void be32(std::vector<uint8_t>& o, int32_t v) {
        for (int i = 0; i < 4; ++i) o.push_back((uint8_t)((uint32_t)v >> (24 - 8 * i)));
    }
    static int64_t rd64(const uint8_t* p) {
        uint64_t v = 0;
        for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
        return (int64_t)v;
    }
    static int32_t rd32(const uint8_t* p) {
        uint32_t v = 0;
        for (int i = 0; i < 4; ++i) v = (v << 8) | p[i];
        return (int32_t)v;
    }
    i128 win_start(i128 k) const { return (i128)cfg.offset + k * (i128)slide(); }

    // Heap-layout snapshot (version 4) of the tumbling / sliding window state: per key group,
    // the reference's "window-contents" entries (window, key, accumulator) -- every (key,
    // window) whose panes hold data, folded, plus the restored windows -- the (empty)
    // merging window set, and the event-time timers (CopyOnWriteStateMapSnapshot.writeState
    // :127-149, TimerSerializer.serialize :147-152, InternalTimerServiceImpl :350-360):
    //   state:   windows not fired yet; under allowed lateness with EventTimeTrigger also the
    //            fired windows that are not cleaned yet (WindowOperator.cleanupTime :670-677);
    //   timers:  maxTimestamp for the windows not fired yet (EventTimeTrigger.onElement),
    //            maxTimestamp + lateness for every window with state when lateness > 0
    //            (registerCleanupTimer :631-643; with lateness 0 the two coincide).
    int snapshot_heap(int32_t kg_lo, int32_t kg_hi, void* buf, int64_t cap, int64_t* len) {
        int rc;
        if (kg_lo < 0 || kg_hi < kg_lo || kg_hi >= cfg.max_parallelism)
            return fail(GW_E_INVALID, "key-group range [%d, %d] outside [0, %d)", kg_lo, kg_hi, cfg.max_parallelism);
        if ((rc = ov_finalize())) return rc;
        if ((rc = ensure_fresh())) return rc;
        if ((rc = flush_buffer())) return rc;  // prepareSnapshotPreBarrier: buffered records first
        if (rf_bound && (rc = process_refire())) return rc;  // late records of fired windows
        if ((rc = refresh())) return rc;
        KhmHost kh;  // keys fed with a key_hash: their key group comes from that hash
        if ((rc = khm_host(kh))) return rc;
        const bool hashed = kh.on();
        auto kg_of = [&](int64_t key) { return key_group_for_hash(kh.hash(key), cfg.max_parallelism); };
        // (key, pane, a0, a1, kg) of every non-null pane cell and parked entry in range
        const int64_t n_def = (int64_t)h_st->n_deferred;
        const int64_t bound = ((int64_t)h_st->used_slots + 1) * popcount(occ) + n_def;
        std::vector<int64_t> col[4];
        std::vector<int32_t> kgs;
        if (bound > 0) {
            int64_t* d = nullptr;
            HIPCHECK(hipMalloc((void**)&d, (size_t)bound * 36));
            SnapArgs a{};
            a.t = tv;
            a.occ = occ;
            for (i128 p = B; p < B + R; ++p) a.pane_of_pos[pos_of(p)] = (int64_t)p;
            a.d_key = dk[cur]; a.d_pane = dp[cur]; a.d_a0 = da0[cur]; a.d_a1 = da1[cur];
            a.n_def = n_def;
            a.max_p = cfg.max_parallelism;
            a.kg_lo = hashed ? 0 : kg_lo;  // hashed keys: every entry, key groups on the host
            a.kg_hi = hashed ? cfg.max_parallelism - 1 : kg_hi;
            a.o_key = d; a.o_pane = d + bound; a.o_a0 = d + 2 * bound; a.o_a1 = d + 3 * bound;
            a.o_kg = (int32_t*)(d + 4 * bound);
            a.n_out = d_tmp + 2;
            hipError_t e = hipMemsetAsync(a.n_out, 0, 8, stream);
            if (e == hipSuccess) e = launch_snap_collect(a, stream);
            unsigned long long n = 0;
            if (e == hipSuccess) e = hipMemcpyAsync(&n, a.n_out, 8, hipMemcpyDeviceToHost, stream);
            if (e == hipSuccess) e = hipStreamSynchronize(stream);
            if (e == hipSuccess) {
                kgs.resize(n);
                for (int c = 0; c < 4 && e == hipSuccess; ++c) {
                    col[c].resize(n);
                    if (n) e = hipMemcpy(col[c].data(), d + c * bound, n * 8, hipMemcpyDeviceToHost);
                }
                if (n && e == hipSuccess) e = hipMemcpy(kgs.data(), a.o_kg, n * 4, hipMemcpyDeviceToHost);
            }
            hipFree(d);
            if (e != hipSuccess) return fail(GW_E_DEVICE, "snapshot: %s", hipGetErrorString(e));
            if (hashed) {  // key groups from the keys' own hashes, then the range filter
                size_t w = 0;
                for (size_t i = 0; i < kgs.size(); ++i) {
                    const int32_t g = kg_of(col[0][i]);
                    if (g < kg_lo || g > kg_hi) continue;
                    for (int c = 0; c < 4; ++c) col[c][w] = col[c][i];
                    kgs[w++] = g;
                }
                kgs.resize(w);
                for (int c = 0; c < 4; ++c) col[c].resize(w);
            }
        }
        // the restored windows still holding state
        std::vector<OvEntry> ov;
        if (ov_n) {
            std::vector<int64_t> oc((size_t)ov_n * 4);
            std::vector<uint32_t> of((size_t)ov_n);
            HIPCHECK(hipMemcpy(oc.data(), d_ov, (size_t)ov_n * 32, hipMemcpyDeviceToHost));
            HIPCHECK(hipMemcpy(of.data(), d_ov_flags, (size_t)ov_n * 4, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < ov_n; ++i) {
                if (of[i] & kOvDead) continue;
                const int32_t kg = kg_of(oc[i]);
                if (kg < kg_lo || kg > kg_hi) continue;
                ov.push_back(OvEntry{oc[i], oc[ov_n + i], oc[2 * ov_n + i], oc[3 * ov_n + i], of[i]});
            }
        }
        const bool lat = cfg.allowed_lateness > 0;
        const bool purging = cfg.trigger == GW_PURGING_EVENT_TIME_TRIGGER;
        const i128 state_lo = (lat && !purging) ? std::min(clean_k_at(wm), fired_k) : fired_k;
        // entries of one key group: panes sorted by (key, pane), overlay by (key, k)
        const int nk = kg_hi - kg_lo + 1;
        std::vector<std::vector<int64_t>> by_kg(nk);  // indices into col
        for (size_t i = 0; i < kgs.size(); ++i) by_kg[kgs[i] - kg_lo].push_back((int64_t)i);
        std::vector<std::vector<OvEntry>> ov_kg(nk);
        for (auto& e : ov) ov_kg[kg_of(e.key) - kg_lo].push_back(e);
        std::vector<uint8_t> pay;
        std::vector<int64_t> offs(nk + 1, 0);
        const int64_t id0 = identity0(cfg.agg);
        const i128 LMAX = INT64_MAX;
        for (int g = 0; g < nk; ++g) {
            offs[g] = (int64_t)pay.size();
            auto& ix = by_kg[g];
            std::sort(ix.begin(), ix.end(), [&](int64_t x, int64_t y) {
                return col[0][x] != col[0][y] ? col[0][x] < col[0][y] : col[1][x] < col[1][y];
            });
            auto& oe = ov_kg[g];
            std::sort(oe.begin(), oe.end(), [](const OvEntry& x, const OvEntry& y) {
                return x.key != y.key ? x.key < y.key : x.k < y.k;
            });
            std::vector<uint8_t> st, tm;
            int32_t nst = 0, ntm = 0;
            size_t a = 0, b = 0;
            while (a < ix.size() || b < oe.size()) {
                // next key
                int64_t key;
                if (a < ix.size() && (b >= oe.size() || col[0][ix[a]] <= oe[b].key)) key = col[0][ix[a]];
                else key = oe[b].key;
                std::vector<std::pair<int64_t, std::pair<int64_t, int64_t>>> panes;  // pane -> cell
                for (; a < ix.size() && col[0][ix[a]] == key; ++a) {
                    const int64_t i = ix[a];
                    if (!panes.empty() && panes.back().first == col[1][i]) {
                        fold_cell(cfg.agg, panes.back().second.first, panes.back().second.second, col[2][i], col[3][i]);
                    } else {
                        panes.push_back({col[1][i], {col[2][i], col[3][i]}});
                    }
                }
                std::vector<OvEntry> ok_;
                for (; b < oe.size() && oe[b].key == key; ++b) ok_.push_back(oe[b]);
                // the windows holding state: those covering a pane with data, and restored ones
                std::vector<i128> ks;
                for (auto& pp : panes) {
                    const i128 p = pp.first;
                    for (i128 k = floor_div(p - (i128)n, (i128)m) + 1; k <= floor_div(p, (i128)m); ++k) ks.push_back(k);
                }
                for (auto& e : ok_) ks.push_back(e.k);
                std::sort(ks.begin(), ks.end());
                ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
                size_t q = 0;
                for (i128 k : ks) {
                    if (k < state_lo) continue;
                    int64_t r0 = id0, r1 = 0;
                    bool any = false;
                    const i128 p0 = k * (i128)m, p1 = p0 + (i128)n;
                    for (auto& pp : panes)
                        if (pp.first >= p0 && pp.first < p1) {
                            fold_cell(cfg.agg, r0, r1, pp.second.first, pp.second.second);
                            any = true;
                        }
                    bool timer = any && k >= fired_k;
                    while (q < ok_.size() && ok_[q].k < k) ++q;
                    if (q < ok_.size() && ok_[q].k == k) {
                        fold_cell(cfg.agg, r0, r1, ok_[q].a0, ok_[q].a1);
                        any = true;
                        if ((ok_[q].flags & kOvTimer) && k >= fired_k) timer = true;
                    }
                    if (!any) continue;
                    const i128 s0 = win_start(k), e0 = s0 + (i128)size();
                    if (!fits64(s0) || !fits64(e0)) return fail(GW_E_RANGE, "window bounds overflow int64");
                    be64(st, (int64_t)s0); be64(st, (int64_t)e0); be64(st, key);
                    if (hashed) be32(st, kh.hash(key));
                    acc_to_be(st, r0, r1);
                    nst++;
                    const i128 mx = e0 - 1;
                    if (timer) {
                        be64(tm, (int64_t)((uint64_t)(int64_t)mx ^ 0x8000000000000000ull));
                        be64(tm, key); be64(tm, (int64_t)s0); be64(tm, (int64_t)e0);
                        ntm++;
                    }
                    const i128 ct = mx + (i128)cfg.allowed_lateness;
                    if (lat && ct < LMAX) {
                        be64(tm, (int64_t)((uint64_t)(int64_t)ct ^ 0x8000000000000000ull));
                        be64(tm, key); be64(tm, (int64_t)s0); be64(tm, (int64_t)e0);
                        ntm++;
                    }
                }
            }
            be32(pay, nst);
            pay.insert(pay.end(), st.begin(), st.end());
            be32(pay, 0);  // merging window set: none for tumbling / sliding windows
            be32(pay, ntm);
            pay.insert(pay.end(), tm.begin(), tm.end());
        }
        offs[nk] = (int64_t)pay.size();
        const int64_t need = (int64_t)sizeof(SnapHeader) + (int64_t)(nk + 1) * 8 + (int64_t)pay.size();
        *len = need;
        if (!buf) return GW_OK;
        if (cap < need) return fail(GW_E_OUTPUT_FULL, "snapshot needs %lld bytes", (long long)need);
        SnapHeader hd{};
        memcpy(hd.magic, "GWS1", 4);
        hd.version = 4;
        hd.agg = cfg.agg; hd.assigner = cfg.assigner;
        hd.size = cfg.size; hd.slide = slide(); hd.offset = cfg.offset; hd.gap = cfg.gap;
        hd.flags = hashed ? kSnapKeyHashes : 0;
        hd.max_parallelism = cfg.max_parallelism; hd.kg_lo = kg_lo; hd.kg_hi = kg_hi;
        hd.entries = (int64_t)pay.size();
        char* out = (char*)buf;
        memcpy(out, &hd, sizeof hd);
        memcpy(out + sizeof hd, offs.data(), (nk + 1) * 8);
        if (!pay.empty()) memcpy(out + sizeof hd + (nk + 1) * 8, pay.data(), pay.size());
        return GW_OK;
    }

    // Restore one heap-layout blob (any key-group range; several calls after rescaling).
    // Only before the first record or watermark, as initializeState runs before processing.
    // The blob is parsed and checked whole (windows, counts, key hashes against each other
    // and against the keys the handle already knows) before anything changes, so a rejected
    // blob leaves the handle as it was; `dry` stops there (composite handles check every
    // class's part before restoring any).
    int restore_heap(const void* buf, int64_t len, bool dry = false) {
        if (!buf || len < (int64_t)sizeof(SnapHeader)) return fail(GW_E_INVALID, "snapshot blob too short");
        SnapHeader hd;
        memcpy(&hd, buf, sizeof hd);
        if (memcmp(hd.magic, "GWS1", 4) != 0 || hd.version < 1 || hd.version > kSnapMaxVersion)
            return fail(GW_E_INVALID, "not a gpuwin snapshot");
        if (hd.version != 4 || hd.agg != cfg.agg || hd.assigner != cfg.assigner || hd.size != cfg.size ||
            hd.slide != slide() || hd.offset != cfg.offset || hd.max_parallelism != cfg.max_parallelism)
            return fail(GW_E_INVALID, "snapshot of a different window / aggregate / max parallelism");
        if (stats.events_in != 0 || wm != INT64_MIN)
            return fail(GW_E_STATE, "restore after processing started (initializeState runs before the first record)");
        const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
        const int64_t pay0 = (int64_t)sizeof hd + (nk + 1) * 8;
        if (nk <= 0 || hd.entries < 0 || len < pay0 || hd.entries > len - pay0) return fail(GW_E_INVALID, "truncated snapshot blob");
        const uint8_t* p = (const uint8_t*)buf + pay0;
        const uint8_t* end = p + hd.entries;
        const int ab = acc_bytes();
        const int hb = (hd.flags & kSnapKeyHashes) ? 4 : 0;
        std::vector<OvEntry> pend;  // the blob's entries, appended to ov_pending once all is checked
        std::vector<int64_t> hkeys;  // (key, hash) of a hashed blob's entries
        std::vector<int32_t> hvals;
        auto by_key_k = [](const OvEntry& x, const OvEntry& y) { return x.key != y.key ? x.key < y.key : x.k < y.k; };
#define NEED(x) do { if ((x) < 0 || (int64_t)(x) > end - p) return fail(GW_E_INVALID, "truncated snapshot blob"); } while (0)
        for (int64_t g = 0; g < nk; ++g) {
            NEED(4);
            const int32_t ns = rd32(p); p += 4;
            if (ns < 0) return fail(GW_E_INVALID, "negative entry count in snapshot key group");
            NEED((int64_t)ns * (24 + hb + ab));
            const size_t base = pend.size();
            for (int32_t i = 0; i < ns; ++i) {
                const int64_t s0 = rd64(p), e0 = rd64(p + 8), key = rd64(p + 16);
                const i128 k = floor_div((i128)s0 - cfg.offset, (i128)slide());
                if (win_start(k) != (i128)s0 || (i128)s0 + size() != (i128)e0)
                    return fail(GW_E_INVALID, "snapshot window [%lld, %lld) is not a window of this assigner",
                                (long long)s0, (long long)e0);
                OvEntry e{key, (int64_t)k, 0, 0, 0};
                if (hb) {
                    hkeys.push_back(key);
                    hvals.push_back(rd32(p + 24));
                }
                acc_from_be(p + 24 + hb, e.a0, e.a1);
                pend.push_back(e);
                p += 24 + hb + ab;
            }
            NEED(4);
            if (rd32(p) != 0) return fail(GW_E_INVALID, "merging window set in a tumbling / sliding snapshot");
            p += 4;
            NEED(4);
            const int32_t nt = rd32(p); p += 4;
            if (nt < 0) return fail(GW_E_INVALID, "negative timer count in snapshot key group");
            NEED((int64_t)nt * 32);
            // an event-time timer at the window's maxTimestamp: the window has not fired
            std::sort(pend.begin() + base, pend.end(), by_key_k);
            for (int32_t i = 0; i < nt; ++i, p += 32) {
                const int64_t ts = (int64_t)((uint64_t)rd64(p) ^ 0x8000000000000000ull);
                const int64_t key = rd64(p + 8), s0 = rd64(p + 16), e0 = rd64(p + 24);
                if (ts != (int64_t)((uint64_t)e0 - 1)) continue;  // cleanup timer: implied by the state
                const int64_t k = (int64_t)floor_div((i128)s0 - cfg.offset, (i128)slide());
                auto it = std::lower_bound(pend.begin() + base, pend.end(), OvEntry{key, k, 0, 0, 0}, by_key_k);
                if (it != pend.end() && it->key == key && it->k == k) it->flags |= kOvTimer;
            }
        }
#undef NEED
        if (p != end) return fail(GW_E_INVALID, "snapshot blob has trailing bytes");
        int rc = khm_check_host(hkeys, hvals);
        if (rc || dry) return rc;
        ov_pending.insert(ov_pending.end(), pend.begin(), pend.end());
        return khm_insert_host(hkeys, hvals);
    }

    // Session windows (blob version 4, the heap layout of snapshot_heap): per key group the
    // "window-contents" entries of the in-flight sessions, the merging window sets and the
    // event-time timers (snapshot_sessions_heap).  Count windows (version 3): per key, the
    // element count and the ring of count-pane accumulators -- the CountTrigger count and
    // the window contents the evicting operator keeps (EvictingWindowOperator.java:92-135).
    uint32_t slot_blob_version() const { return cfg.assigner == GW_COUNT_SLIDING ? 3u : 4u; }

    // countWindow(size) = GlobalWindows + PurgingTrigger(CountTrigger(size)) (KeyedStream.java:
    // 676-678) in the heap layout (blob version 4, as oracle/flink_oracle.c count_snapshot):
    // per key group "window-contents" = be32 n; n x (GlobalWindow = one byte 0, key, [be32
    // hash,] state) -- the fold of the key's elements since its last FIRE_AND_PURGE, i.e. the
    // current count pane (a tumbling count window is one pane); "count" = be32 n; n x (byte 0,
    // key, [be32 hash,] be64 c mod size) -- CountTrigger's ReducingState<Long>
    // (CountTrigger.java:39-40); be32 0 timers (GlobalWindow ends at Long.MAX_VALUE: no cleanup
    // timer; CountTrigger registers none).  A key whose element count is a multiple of size
    // was just purged and holds no state.  The sliding form keeps the version-3 layout.
    int snapshot_count_heap(int32_t kg_lo, int32_t kg_hi, void* buf, int64_t cap, int64_t* len) {
        int rc;
        if ((rc = session_refresh(sess, err))) return fail(rc, "%s", err.c_str());
        KhmHost kh;
        if ((rc = khm_host(kh))) return rc;
        const bool hashed = kh.on();
        std::vector<int64_t> ent;
        std::vector<int32_t> kgs;
        if ((rc = session_collect(sess, kg_lo, kg_hi, ent, kgs, err,
                                  hashed ? std::function<int32_t(int64_t)>([&](int64_t k) { return kh.hash(k); })
                                         : std::function<int32_t(int64_t)>())))
            return fail(rc, "%s", err.c_str());
        const int64_t ew = session_entry_words(sess), W = tv.words;
        const int64_t ring = (ew - 2) / W;
        const int nk = kg_hi - kg_lo + 1;
        std::vector<std::vector<int64_t>> by_kg(nk);
        for (size_t i = 0; i < kgs.size(); ++i) {
            const int64_t c = ent[ew * i + 1];
            if (c % cfg.size != 0) by_kg[kgs[i] - kg_lo].push_back((int64_t)i);
        }
        std::vector<uint8_t> pay;
        std::vector<int64_t> offs(nk + 1, 0);
        for (int g = 0; g < nk; ++g) {
            offs[g] = (int64_t)pay.size();
            auto& ix = by_kg[g];
            std::sort(ix.begin(), ix.end(), [&](int64_t x, int64_t y) { return ent[ew * x] < ent[ew * y]; });
            std::vector<uint8_t> cnt;
            be32(pay, (int32_t)ix.size());
            be32(cnt, (int32_t)ix.size());
            for (int64_t i : ix) {
                const int64_t* e = &ent[ew * i];
                const int64_t key = e[0], c = e[1];
                const int64_t* cell = e + 2 + (((c - 1) / cfg.size) % ring) * W;  // the current count pane
                pay.push_back(0);
                be64(pay, key);
                if (hashed) be32(pay, kh.hash(key));
                acc_to_be(pay, cell[0], W == 2 ? cell[1] : 0);
                cnt.push_back(0);
                be64(cnt, key);
                if (hashed) be32(cnt, kh.hash(key));
                be64(cnt, c % cfg.size);
            }
            pay.insert(pay.end(), cnt.begin(), cnt.end());
            be32(pay, 0);
        }
        offs[nk] = (int64_t)pay.size();
        const int64_t need = (int64_t)sizeof(SnapHeader) + (int64_t)(nk + 1) * 8 + (int64_t)pay.size();
        *len = need;
        if (!buf) return GW_OK;
        if (cap < need) return fail(GW_E_OUTPUT_FULL, "snapshot needs %lld bytes", (long long)need);
        SnapHeader hd{};
        memcpy(hd.magic, "GWS1", 4);
        hd.version = 4;
        hd.agg = cfg.agg; hd.assigner = cfg.assigner;
        hd.size = cfg.size; hd.slide = cfg.slide; hd.offset = cfg.offset; hd.gap = cfg.gap;
        hd.flags = hashed ? kSnapKeyHashes : 0;
        hd.max_parallelism = cfg.max_parallelism; hd.kg_lo = kg_lo; hd.kg_hi = kg_hi;
        hd.entries = (int64_t)pay.size();
        char* out = (char*)buf;
        memcpy(out, &hd, sizeof hd);
        memcpy(out + sizeof hd, offs.data(), (nk + 1) * 8);
        if (!pay.empty()) memcpy(out + sizeof hd + (nk + 1) * 8, pay.data(), pay.size());
        return GW_OK;
    }
    // ... and back into version-3 entries (key, element count = the trigger's count, the
    // contents in count pane 0 of the ring, identities elsewhere)
    int parse_count_heap(const SnapHeader& hd, const uint8_t* p, const uint8_t* end, std::vector<int64_t>& ent,
                         std::vector<int64_t>& hkeys, std::vector<int32_t>& hvals) {
        const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
        const int hb = (hd.flags & kSnapKeyHashes) ? 4 : 0, ab = acc_bytes();
        const int64_t ew = session_entry_words(sess), W = tv.words;
#define NEED(x) do { if ((int64_t)(x) > end - p) return fail(GW_E_INVALID, "truncated snapshot blob"); } while (0)
        for (int64_t g = 0; g < nk; ++g) {
            NEED(4);
            const int32_t n = rd32(p);
            p += 4;
            if (n < 0) return fail(GW_E_INVALID, "corrupt snapshot blob");
            NEED((int64_t)n * (9 + hb + ab));
            const uint8_t* st = p;
            p += (int64_t)n * (9 + hb + ab);
            NEED(4);
            const int32_t m = rd32(p);
            p += 4;
            if (m != n) return fail(GW_E_INVALID, "count-window contents without their CountTrigger count");
            NEED((int64_t)m * (17 + hb));
            for (int32_t i = 0; i < n; ++i) {
                const uint8_t* x = st + (int64_t)i * (9 + hb + ab);
                const uint8_t* c = p + (int64_t)i * (17 + hb);
                const int64_t key = rd64(x + 1), cnt = rd64(c + 9 + hb);
                if (x[0] != 0 || c[0] != 0 || rd64(c + 1) != key || cnt <= 0 || cnt >= cfg.size)
                    return fail(GW_E_INVALID, "corrupt count-window snapshot entry");
                if (hb) { hkeys.push_back(key); hvals.push_back(rd32(x + 9)); }
                const size_t at = ent.size();
                ent.resize(at + (size_t)ew, 0);
                ent[at] = key;
                ent[at + 1] = cnt;
                for (int64_t q = 2; q < ew; q += W) {  // identities, then the contents in pane 0
                    ent[at + q] = identity0(cfg.agg);
                    if (W == 2) ent[at + q + 1] = 0;
                }
                int64_t a0, a1;
                acc_from_be(x + 9 + hb, a0, a1);
                ent[at + 2] = a0;
                if (W == 2) ent[at + 3] = a1;
            }
            p += (int64_t)m * (17 + hb);
            NEED(4);
            if (rd32(p) != 0) return fail(GW_E_INVALID, "count windows hold no timers");
            p += 4;
        }
#undef NEED
        if (p != end) return fail(GW_E_INVALID, "snapshot blob has trailing bytes");
        return GW_OK;
    }

    // Session windows in the heap backend's layout (HeapSnapshotStrategy.java:97-154), per key
    // group and big-endian like snapshot_heap:
    //   "window-contents": be32 n; n x (state window, key, [be32 key hash,] accumulator): one
    //       entry per in-flight session holding state (CopyOnWriteStateMapSnapshot.writeState
    //       :127-149).  The GPU keeps a session's state under the session itself, so its state
    //       window is the window; a fired session under PurgingTrigger holds no state (its
    //       contents were purged, WindowOperator.java:482-484) and has no entry;
    //   "merging-window-set": be32 m; m x (key, [be32 key hash,] be32 c, c x (window, state
    //       window)): the key's MergingWindowSet mapping (MergingWindowSet.persist :99-106);
    //   timers: be32 t; t x (flipSignBit(ts), key, window) (TimerSerializer :147-152): the
    //       trigger's timer at maxTimestamp while the session has not fired
    //       (EventTimeTrigger.onElement / onMerge) and, under allowed lateness, its cleanup
    //       timer (registerCleanupTimer :631-643; with lateness 0 the two coincide).
    // Order: keys ascending, a key's sessions by start, its timers by (window, time).
    int snapshot_sessions_heap(int32_t kg_lo, int32_t kg_hi, void* buf, int64_t cap, int64_t* len) {
        int rc;
        if ((rc = session_refresh(sess, err))) return fail(rc, "%s", err.c_str());
        KhmHost kh;
        if ((rc = khm_host(kh))) return rc;
        const bool hashed = kh.on();
        std::vector<int64_t> ent;  // (key, start, end, a0, a1, fired) per session
        std::vector<int32_t> kgs;
        if ((rc = session_collect(sess, kg_lo, kg_hi, ent, kgs, err,
                                  hashed ? std::function<int32_t(int64_t)>([&](int64_t k) { return kh.hash(k); })
                                         : std::function<int32_t(int64_t)>())))
            return fail(rc, "%s", err.c_str());
        const int nk = kg_hi - kg_lo + 1;
        std::vector<std::vector<int64_t>> by_kg(nk);
        for (size_t i = 0; i < kgs.size(); ++i) by_kg[kgs[i] - kg_lo].push_back((int64_t)i);
        const bool purging = cfg.trigger == GW_PURGING_EVENT_TIME_TRIGGER;
        const i128 LMAX = INT64_MAX;
        std::vector<uint8_t> pay;
        std::vector<int64_t> offs(nk + 1, 0);
        for (int g = 0; g < nk; ++g) {
            offs[g] = (int64_t)pay.size();
            auto& ix = by_kg[g];
            std::sort(ix.begin(), ix.end(), [&](int64_t x, int64_t y) {
                const int64_t* a = &ent[6 * x];
                const int64_t* b = &ent[6 * y];
                return a[0] != b[0] ? a[0] < b[0] : a[1] < b[1];
            });
            std::vector<uint8_t> st, ms, tm;
            int32_t nst = 0, nms = 0, ntm = 0;
            for (size_t a = 0; a < ix.size();) {
                const int64_t key = ent[6 * ix[a]];
                size_t b = a;
                while (b < ix.size() && ent[6 * ix[b]] == key) ++b;
                be64(ms, key);
                if (hashed) be32(ms, kh.hash(key));
                be32(ms, (int32_t)(b - a));
                nms++;
                for (size_t q = a; q < b; ++q) {
                    const int64_t* x = &ent[6 * ix[q]];
                    const int64_t s0 = x[1], e0 = x[2];
                    const bool fired = x[5] != 0;
                    be64(ms, s0); be64(ms, e0); be64(ms, s0); be64(ms, e0);
                    if (!(purging && fired)) {
                        be64(st, s0); be64(st, e0); be64(st, key);
                        if (hashed) be32(st, kh.hash(key));
                        acc_to_be(st, x[3], x[4]);
                        nst++;
                    }
                    const i128 mx = (i128)e0 - 1;
                    if (!fired) {
                        be64(tm, (int64_t)((uint64_t)(int64_t)mx ^ 0x8000000000000000ull));
                        be64(tm, key); be64(tm, s0); be64(tm, e0);
                        ntm++;
                    }
                    const i128 ct = mx + (i128)cfg.allowed_lateness;
                    if (cfg.allowed_lateness > 0 && ct < LMAX) {
                        be64(tm, (int64_t)((uint64_t)(int64_t)ct ^ 0x8000000000000000ull));
                        be64(tm, key); be64(tm, s0); be64(tm, e0);
                        ntm++;
                    }
                }
                a = b;
            }
            be32(pay, nst);
            pay.insert(pay.end(), st.begin(), st.end());
            be32(pay, nms);
            pay.insert(pay.end(), ms.begin(), ms.end());
            be32(pay, ntm);
            pay.insert(pay.end(), tm.begin(), tm.end());
        }
        offs[nk] = (int64_t)pay.size();
        const int64_t need = (int64_t)sizeof(SnapHeader) + (int64_t)(nk + 1) * 8 + (int64_t)pay.size();
        *len = need;
        if (!buf) return GW_OK;
        if (cap < need) return fail(GW_E_OUTPUT_FULL, "snapshot needs %lld bytes", (long long)need);
        SnapHeader hd{};
        memcpy(hd.magic, "GWS1", 4);
        hd.version = 4;
        hd.agg = cfg.agg; hd.assigner = cfg.assigner;
        hd.size = cfg.size; hd.slide = cfg.slide; hd.offset = cfg.offset; hd.gap = cfg.gap;
        hd.flags = hashed ? kSnapKeyHashes : 0;
        hd.max_parallelism = cfg.max_parallelism; hd.kg_lo = kg_lo; hd.kg_hi = kg_hi;
        hd.entries = (int64_t)pay.size();
        char* out = (char*)buf;
        memcpy(out, &hd, sizeof hd);
        memcpy(out + sizeof hd, offs.data(), (nk + 1) * 8);
        if (!pay.empty()) memcpy(out + sizeof hd + (nk + 1) * 8, pay.data(), pay.size());
        return GW_OK;
    }

    // Reads a session blob of the heap layout back into (key, start, end, a0, a1, fired)
    // sessions: each merging-window-set mapping (window -> state window) takes the state of
    // its state window (any original window, as the reference's MergingWindowSet.addWindow
    // keeps it, :188-201), or none; a session has fired when its trigger timer at
    // maxTimestamp is gone.  A session without state that has not fired is a trigger outside
    // EventTimeTrigger / PurgingTrigger (GW_E_UNSUPPORTED); state no mapping names, or
    // overlapping sessions of one key, are a corrupt blob.
    int parse_session_heap(const SnapHeader& hd, const uint8_t* p, const uint8_t* end, std::vector<int64_t>& out,
                           std::vector<int64_t>& hkeys, std::vector<int32_t>& hvals) {
        const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
        const int ab = acc_bytes();
        const int hb = (hd.flags & kSnapKeyHashes) ? 4 : 0;
        const int64_t id0 = cfg.agg == GW_AVG_F64 ? INT64_MIN : identity0(cfg.agg);  // a purged session
        typedef std::tuple<int64_t, int64_t, int64_t> KW;  // (key, start, end)
#define NEED(x) do { if ((x) < 0 || (int64_t)(x) > end - p) return fail(GW_E_INVALID, "truncated snapshot blob"); } while (0)
        for (int64_t g = 0; g < nk; ++g) {
            NEED(4);
            const int32_t ns = rd32(p); p += 4;
            if (ns < 0) return fail(GW_E_INVALID, "negative entry count in snapshot key group");
            NEED((int64_t)ns * (24 + hb + ab));
            std::map<KW, std::pair<std::pair<int64_t, int64_t>, bool>> state;  // -> (acc, used)
            for (int32_t i = 0; i < ns; ++i, p += 24 + hb + ab) {
                const int64_t s0 = rd64(p), e0 = rd64(p + 8), key = rd64(p + 16);
                int64_t a0, a1;
                acc_from_be(p + 24 + hb, a0, a1);
                if (hb) { hkeys.push_back(key); hvals.push_back(rd32(p + 24)); }
                if (!state.emplace(KW{key, s0, e0}, std::make_pair(std::make_pair(a0, a1), false)).second)
                    return fail(GW_E_INVALID, "two state entries of one (key, window) in a snapshot key group");
            }
            NEED(4);
            const int32_t nm = rd32(p); p += 4;
            if (nm < 0) return fail(GW_E_INVALID, "negative merging window set count in snapshot key group");
            std::vector<std::array<int64_t, 5>> ses;  // (key, start, end, state start, state end)
            for (int32_t i = 0; i < nm; ++i) {
                NEED(12 + hb);
                const int64_t key = rd64(p);
                if (hb) { hkeys.push_back(key); hvals.push_back(rd32(p + 8)); }
                const int32_t c = rd32(p + 8 + hb);
                p += 12 + hb;
                if (c < 0) return fail(GW_E_INVALID, "negative merging window set size");
                NEED((int64_t)c * 32);
                for (int32_t j = 0; j < c; ++j, p += 32)
                    ses.push_back({key, rd64(p), rd64(p + 8), rd64(p + 16), rd64(p + 24)});
            }
            NEED(4);
            const int32_t nt = rd32(p); p += 4;
            if (nt < 0) return fail(GW_E_INVALID, "negative timer count in snapshot key group");
            NEED((int64_t)nt * 32);
            std::set<KW> armed;  // sessions whose trigger timer (at maxTimestamp) is still set
            for (int32_t i = 0; i < nt; ++i, p += 32) {
                const int64_t ts = (int64_t)((uint64_t)rd64(p) ^ 0x8000000000000000ull);
                const int64_t key = rd64(p + 8), s0 = rd64(p + 16), e0 = rd64(p + 24);
                if (ts == (int64_t)((uint64_t)e0 - 1)) armed.insert(KW{key, s0, e0});
            }
            std::sort(ses.begin(), ses.end());
            for (size_t i = 0; i < ses.size(); ++i) {
                const auto& x = ses[i];
                if (x[2] <= x[1]) return fail(GW_E_INVALID, "empty session window in a snapshot");
                if (i && ses[i - 1][0] == x[0] && ses[i - 1][2] >= x[1])  // TimeWindow.intersects is inclusive
                    return fail(GW_E_INVALID, "overlapping sessions of one key in a snapshot");
                const bool fired = armed.count(KW{x[0], x[1], x[2]}) == 0;
                auto it = state.find(KW{x[0], x[3], x[4]});
                int64_t a0 = id0, a1 = 0;
                if (it != state.end()) {
                    if (it->second.second) return fail(GW_E_INVALID, "two sessions share one state window");
                    it->second.second = true;
                    a0 = it->second.first.first;
                    a1 = it->second.first.second;
                } else if (!fired) {
                    return fail(GW_E_UNSUPPORTED, "a session without state whose timer has not fired "
                                                  "(a trigger other than EventTimeTrigger / PurgingTrigger)");
                }
                out.insert(out.end(), {x[0], x[1], x[2], a0, a1, (int64_t)fired});
            }
            for (auto& kv : state)
                if (!kv.second.second) return fail(GW_E_INVALID, "a state entry outside every merging window set");
        }
#undef NEED
        if (p != end) return fail(GW_E_INVALID, "snapshot blob has trailing bytes");
        return GW_OK;
    }

    int snapshot_sessions(int32_t kg_lo, int32_t kg_hi, void* buf, int64_t cap, int64_t* len) {
        int rc;
        if (kg_lo < 0 || kg_hi < kg_lo || kg_hi >= cfg.max_parallelism)
            return fail(GW_E_INVALID, "key-group range [%d, %d] outside [0, %d)", kg_lo, kg_hi, cfg.max_parallelism);
        if (cfg.assigner == GW_SESSION) return snapshot_sessions_heap(kg_lo, kg_hi, buf, cap, len);
        if (cfg.assigner == GW_COUNT_TUMBLING) return snapshot_count_heap(kg_lo, kg_hi, buf, cap, len);
        if ((rc = session_refresh(sess, err))) return fail(rc, "%s", err.c_str());
        KhmHost kh;
        if ((rc = khm_host(kh))) return rc;
        const bool hashed = kh.on();
        std::vector<int64_t> ent;
        std::vector<int32_t> kgs;
        if ((rc = session_collect(sess, kg_lo, kg_hi, ent, kgs, err,
                                  hashed ? std::function<int32_t(int64_t)>([&](int64_t k) { return kh.hash(k); })
                                         : std::function<int32_t(int64_t)>())))
            return fail(rc, "%s", err.c_str());
        const int64_t ew0 = session_entry_words(sess);
        if (hashed) {  // each entry gets the key's hash as one more word
            std::vector<int64_t> w;
            w.reserve(ent.size() / ew0 * (ew0 + 1));
            for (size_t i = 0; i < ent.size(); i += ew0) {
                w.insert(w.end(), ent.begin() + i, ent.begin() + i + ew0);
                w.push_back((int64_t)kh.hash(ent[i]));
            }
            ent.swap(w);
        }
        const int64_t ew = ew0 + (hashed ? 1 : 0);
        const int nk = kg_hi - kg_lo + 1;
        std::vector<int64_t> offs(nk + 1, 0);
        for (int32_t k : kgs) offs[k - kg_lo + 1]++;
        for (int i = 0; i < nk; ++i) offs[i + 1] += offs[i];
        const int64_t need = (int64_t)sizeof(SnapHeader) + (int64_t)(nk + 1) * 8 + (int64_t)kgs.size() * ew * 8;
        *len = need;
        if (!buf) return GW_OK;
        if (cap < need) return fail(GW_E_OUTPUT_FULL, "snapshot needs %lld bytes", (long long)need);
        SnapHeader hd{};
        memcpy(hd.magic, "GWS1", 4);
        hd.version = slot_blob_version();
        hd.agg = cfg.agg; hd.assigner = cfg.assigner;
        hd.size = cfg.size; hd.slide = cfg.slide; hd.gap = cfg.gap;
        hd.max_parallelism = cfg.max_parallelism; hd.kg_lo = kg_lo; hd.kg_hi = kg_hi;
        hd.reserved = (int32_t)ew;
        hd.flags = hashed ? kSnapKeyHashes : 0;
        hd.entries = (int64_t)kgs.size();
        char* out = (char*)buf;
        memcpy(out, &hd, sizeof hd);
        memcpy(out + sizeof hd, offs.data(), (nk + 1) * 8);
        int64_t* oe = (int64_t*)(out + sizeof hd + (nk + 1) * 8);
        std::vector<int64_t> fill(offs.begin(), offs.end() - 1);
        for (size_t i = 0; i < kgs.size(); ++i) memcpy(oe + ew * fill[kgs[i] - kg_lo]++, &ent[ew * i], ew * 8);
        return GW_OK;
    }

    int restore_sessions(const void* buf, int64_t len, bool dry = false) {
        if (!buf || len < (int64_t)sizeof(SnapHeader)) return fail(GW_E_INVALID, "snapshot blob too short");
        SnapHeader hd;
        memcpy(&hd, buf, sizeof hd);
        if (memcmp(hd.magic, "GWS1", 4) != 0 || hd.version < 1 || hd.version > kSnapMaxVersion)
            return fail(GW_E_INVALID, "not a gpuwin snapshot");
        if (cfg.assigner == GW_SESSION) {
            if (hd.version != 4 || hd.agg != cfg.agg || hd.assigner != cfg.assigner || hd.gap != cfg.gap ||
                hd.max_parallelism != cfg.max_parallelism || (hd.flags & ~kSnapKeyHashes))
                return fail(GW_E_INVALID, "snapshot of a different window / aggregate / max parallelism");
            const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
            const int64_t pay0 = (int64_t)sizeof hd + (nk + 1) * 8;
            if (nk <= 0 || hd.entries < 0 || len < pay0 || hd.entries > len - pay0)
                return fail(GW_E_INVALID, "truncated snapshot blob");
            const uint8_t* p = (const uint8_t*)buf + pay0;
            std::vector<int64_t> ent, hkeys;
            std::vector<int32_t> hvals;
            int rc = parse_session_heap(hd, p, p + hd.entries, ent, hkeys, hvals);
            if (rc == GW_OK) rc = khm_check_host(hkeys, hvals);  // before the table changes
            if (rc || dry) return rc;
            rc = session_restore(sess, ent.data(), (int64_t)(ent.size() / 6), err);
            if (rc) return fail(rc, "%s", err.c_str());
            return khm_insert_host(hkeys, hvals);
        }
        if (cfg.assigner == GW_COUNT_TUMBLING) {
            if (hd.version != 4 || hd.agg != cfg.agg || hd.assigner != cfg.assigner || hd.size != cfg.size ||
                hd.max_parallelism != cfg.max_parallelism || (hd.flags & ~kSnapKeyHashes))
                return fail(GW_E_INVALID, "snapshot of a different window / aggregate / max parallelism");
            const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
            const int64_t pay0 = (int64_t)sizeof hd + (nk + 1) * 8;
            if (nk <= 0 || hd.entries < 0 || len < pay0 || hd.entries > len - pay0)
                return fail(GW_E_INVALID, "truncated snapshot blob");
            const uint8_t* p = (const uint8_t*)buf + pay0;
            std::vector<int64_t> ent, hkeys;
            std::vector<int32_t> hvals;
            int rc = parse_count_heap(hd, p, p + hd.entries, ent, hkeys, hvals);
            if (rc == GW_OK) rc = khm_check_host(hkeys, hvals);
            if (rc || dry) return rc;
            rc = session_restore(sess, ent.data(), (int64_t)(ent.size() / session_entry_words(sess)), err);
            if (rc) return fail(rc, "%s", err.c_str());
            return khm_insert_host(hkeys, hvals);
        }
        const bool hashed = (hd.flags & kSnapKeyHashes) != 0;
        const int64_t ew0 = session_entry_words(sess), ew = ew0 + (hashed ? 1 : 0);
        if (hd.version != slot_blob_version() || hd.agg != cfg.agg || hd.assigner != cfg.assigner ||
            hd.gap != cfg.gap || hd.size != cfg.size || hd.slide != cfg.slide ||
            hd.max_parallelism != cfg.max_parallelism || hd.reserved != (int32_t)ew)
            return fail(GW_E_INVALID, "snapshot of a different window / aggregate / max parallelism");
        const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
        const int64_t hdr = (int64_t)sizeof hd + (nk + 1) * 8;
        if (nk <= 0 || hd.entries < 0 || len < hdr || hd.entries > (len - hdr) / (ew * 8))
            return fail(GW_E_INVALID, "truncated snapshot blob");
        const int64_t* in = (const int64_t*)((const char*)buf + hdr);
        std::vector<int64_t> ent, hkeys;
        std::vector<int32_t> hvals;
        ent.reserve((size_t)(hd.entries * ew0));
        for (int64_t i = 0; i < hd.entries; ++i) {  // aligned copy without the hash words
            const size_t at = ent.size();
            ent.resize(at + (size_t)ew0);
            memcpy(ent.data() + at, (const char*)in + i * ew * 8, (size_t)ew0 * 8);
            if (hashed) {
                int64_t hw;
                memcpy(&hw, (const char*)in + (i * ew + ew0) * 8, 8);
                hkeys.push_back(ent[at]);
                hvals.push_back((int32_t)hw);
            }
        }
        int rc = khm_check_host(hkeys, hvals);  // before the table changes
        if (rc || dry) return rc;
        rc = session_restore(sess, ent.data(), hd.entries, err);
        if (rc) return fail(rc, "%s", err.c_str());
        return khm_insert_host(hkeys, hvals);
    }

#ifndef GW_FAST_FIRE
#define GW_FAST_FIRE 1  // 0: every fire after a flush waits for the flush's status first
#endif
    int64_t fast_fires = 0;  // fires enqueued behind their flush (gw_kernel_time_ms which = 3)
    // The common fire -- no lateness, no restored windows, nothing deferred, one pass of
    // windows starting at fired_k -- enqueued right behind the flush that precedes it, with
    // k_fire_guard between them: ONE host round trip per watermark instead of two (the flush's
    // status refresh and the fire's).  Everything the fire needs is decided on the host
    // without the flush's counters: k_first = fired_k holds whenever the lowest pane the host
    // knows of in the ring gives no later start (the device's ring holds at least those
    // panes), no ring position is evicted (k_first * m >= B), and the ring reaches k_target.
    // What the host would have read -- spills, wide records, a full table, a deferred entry,
    // the row buffer's room -- the guard reads on the device; when any of them would have
    // changed the host's course the fire does nothing (fire_skip), the flush is finished the
    // exact way (flush_post) and advance_pane goes on as before.  done: the fire ran.
    // Measured (profiles/r6/fastfire/): the flush->fire gap of the headline's fire cycle.
    int fast_fire(i128 kt, uint64_t need, bool& done) {
        done = false;
        int rc;
        const bool eligible = GW_FAST_FIRE && ov_n == 0 && !rf_bound && occ != 0 && h_st->n_deferred == 0;
        const i128 k_first = fired_k;
        if (eligible) {
            const i128 kl = floor_div(ring_min() - n, m) + 1;
            if (kl > k_first || k_first * m < B || floor_div(k_first * m + R - n, m) < kt) return flush_buffer(need);
        } else {
            return flush_buffer(need);
        }
        PendingFlush pf;
        bool launched = false;
        if ((rc = flush_launch(need, pf, launched))) return rc;
        const i128 B0 = B;
        const uint64_t stale0 = stale_pos;
        B = k_first * m;  // rebase(k_first * m) without an eviction
        FireArgs f{};
        i128 keep;
        if ((rc = fire_args(k_first, kt, (kt + 1) * m, f, keep))) return rc;
        f.o_key = o_key; f.o_start = o_start; f.o_end = o_end; f.o_res = o_res;
        f.guarded = 1;
        lazy_retire(f);
        FireGuard g{0, o_cap, (int64_t)f.nwin, rows_reset_pending ? 1 : 0};
        rows_reset_pending = false;  // the guard zeroes the cursor
        HIPCHECK(launch_fire_guard(d_st, g, stream));
        if ((rc = fire_launch(f))) return rc;
        dirty = true;
        if ((rc = refresh())) return rc;
        if (!h_st->fire_skip) {
            fired(f, kt, keep);
            dirty = false;  // the refresh above followed the fire
            occ = h_st->occ;
            fast_fires++;
            done = true;
            return GW_OK;
        }
        // the fire did nothing: undo the host's side of it and take the exact path
        B = B0;
        stale_pos = stale0;
        if (timing) t_fire.drop_last();
        return launched ? flush_post(pf) : GW_OK;
    }

    int advance_pane(int64_t w, int64_t* rows_out) {
        int rc;
        if (rows_out) *rows_out = 0;
        if (w <= wm) return GW_OK;
        if ((rc = ov_finalize())) return rc;
        const i128 kt = k_for_wm(w);
        const i128 ct = clean_k_at(w);
        int64_t before = 0;
        if (cfg.allowed_lateness > 0) {
            if ((rc = ensure_fresh())) return rc;
            before = (int64_t)h_st->rows;
            // rows of the interval's late records come before the timers' rows
            if (rf_bound && (rc = process_refire())) return rc;
            if (kt < fired_k && !(occ && ct * m > B)) {  // nothing fires, nothing is cleaned
                wm = w;
                if ((rc = ensure_fresh())) return rc;
                const int64_t fired = (int64_t)h_st->rows - before;
                stats.rows_fired += fired;
                if (rows_out) *rows_out = fired;
                return GW_OK;
            }
        } else {
            if (kt < fired_k) {  // no window completes: nothing to launch (timer heap empty below w)
                wm = w;
                return GW_OK;
            }
            // buffered records first, then the timers; the flush ends with a status refresh
            // (and emits no row), so the row count before the firing is read after it: one
            // host round trip fewer per fire than a refresh before the flush.  Only the ring
            // positions of panes up to the last one of the last window firing now must be
            // applied; newer panes may wait for the next flush (nar2 carry).
            uint64_t need = ~0ull;
            const i128 plast = kt * m + n - 1;
            if (plast < B + R - 1) {
                need = 0;
                for (i128 P = B; P <= plast; ++P) need |= 1ull << pos_of(P);
            }
            bool done = false;
            if ((rc = fast_fire(kt, need, done))) return rc;
            if (done) {
                wm = w;
                const int64_t fired_rows = (int64_t)h_st->rows - (int64_t)h_st->fire_rows0;
                stats.rows_fired += fired_rows;
                if (rows_out) *rows_out = fired_rows;
                return GW_OK;
            }
            if ((rc = ensure_fresh())) return rc;
            before = (int64_t)h_st->rows;
        }
        // buffered records first, then the timers (without lateness only the positions the
        // firing needs were applied above; the rest stays carried for the next flush)
        if (cfg.allowed_lateness > 0 && (rc = flush_buffer())) return rc;
        {
            if ((rc = fire_until(kt, ct))) return rc;
            wm = w;
        }
        if ((rc = ensure_fresh())) return rc;
        const int64_t fired = (int64_t)h_st->rows - before;
        stats.rows_fired += fired;
        if (rows_out) *rows_out = fired;
        ov_maybe_release(w);
        return GW_OK;
    }
};

// ------------------------------------------------------------------------- ABI
extern "C" {

int gw_abi_version(void) { return GW_ABI_VERSION; }

const char* gw_last_error(const gw_handle* h) {
    if (!h) return g_create_error.c_str();
    return h->err.c_str();
}

static int validate(const gw_config* c, std::string& why) {
    auto ab = [](int64_t v) { return v < 0 ? -v : v; };
    if (c->assigner == GW_TUMBLING) {
        if (c->size <= 0 || ab(c->offset) >= c->size) {
            why = "TumblingEventTimeWindows parameters must satisfy abs(offset) < size";
            return GW_E_INVALID;
        }
    } else if (c->assigner == GW_SLIDING) {
        if (c->slide <= 0 || ab(c->offset) >= c->slide || c->size <= 0) {
            why = "SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0";
            return GW_E_INVALID;
        }
        if (c->size / c->slide > 10000000) {
            why = "SlidingEventTimeWindows parameters must satisfy size / slide <= 10000000";
            return GW_E_INVALID;
        }
    } else if (c->assigner == GW_SESSION) {
        if (c->gap <= 0) {
            why = "EventTimeSessionWindows parameters must satisfy 0 < size";
            return GW_E_INVALID;
        }
    } else if (c->assigner == GW_COUNT_TUMBLING || c->assigner == GW_COUNT_SLIDING) {
        const int64_t slide = c->assigner == GW_COUNT_SLIDING ? c->slide : c->size;
        if (c->size <= 0 || slide <= 0) {
            why = "count windows need size > 0 and slide > 0";
            return GW_E_INVALID;
        }
        int64_t a = c->size, b = slide;
        while (b) { const int64_t t = a % b; a = b; b = t; }
        if (c->size / a > 4096) {
            why = "count window size / gcd(size, slide) > 4096 panes is not supported on the GPU path";
            return GW_E_UNSUPPORTED;
        }
    } else {
        why = "unknown window assigner";
        return GW_E_INVALID;
    }
    if (c->allowed_lateness < 0) { why = "The allowed lateness cannot be negative."; return GW_E_INVALID; }
    if (c->agg < GW_COUNT || c->agg > GW_SUM_I32) { why = "unknown aggregate"; return GW_E_INVALID; }
    if (c->trigger != GW_EVENT_TIME_TRIGGER && c->trigger != GW_PURGING_EVENT_TIME_TRIGGER) {
        why = "unknown trigger";
        return GW_E_INVALID;
    }
    return GW_OK;
}

// Ring positions a sliding (or tumbling: slide = size) assigner needs: the n panes of the
// oldest unfired window + at least one slide ahead, plus, with allowed lateness, the panes
// of fired windows kept until their cleanup (ceil(lateness / slide) + 1 more slides).
// Pane geometry (width g, n panes per window, m per slide): g = gcd(size, slide), except for
// size < slide, where a pane is one slide with the window at its start and the rest a gap.
static void pane_geometry(int64_t size, int64_t slide, int64_t& g, int64_t& n, int64_t& m) {
    if (size < slide) {
        g = slide; n = 1; m = 1;
    } else {
        g = gcd64(size, slide); n = size / g; m = slide / g;
    }
}
static int64_t ring_need(int64_t size, int64_t slide, int64_t lateness) {
    int64_t g, n, m;
    pane_geometry(size, slide, g, n, m);
    if (n > kMaxRing || m > kMaxRing) return kMaxRing + 1;
    int64_t need = n + std::max<int64_t>(m, 1);
    if (lateness > 0) {
        const int64_t extra = lateness / slide + 2;
        if (extra > kMaxRing || need + extra * m > kMaxRing) return kMaxRing + 1;
        need += extra * m;
    }
    return need;
}
// The fewest window classes J whose assigner (size, J * slide) fits the ring, 0 if none
// below 4096 does (or J * slide overflows).
static int64_t class_count(int64_t size, int64_t slide, int64_t lateness) {
    for (int64_t J = 2; J <= 4096; ++J) {
        if (slide > INT64_MAX / J) return 0;
        if (ring_need(size, slide * J, lateness) <= kMaxRing) return J;
    }
    return 0;
}
// A composite handle h (its cfg set): J children on child 0's stream.  Tumbling windows split
// the same way: class j is a sliding assigner (size, J * size, offset + j * size).
static int make_composite(gw_handle* h, int64_t J) {
    gw_config c = h->cfg;
    if (c.assigner == GW_TUMBLING) {
        c.assigner = GW_SLIDING;
        c.slide = c.size;
    }
    if (h->stream) {  // the composite launches nothing of its own
        hipStreamSynchronize(h->stream);
        hipStreamDestroy(h->stream);
        h->stream = nullptr;
    }
    for (int64_t j = 0; j < J; ++j) {
        gw_config k = c;
        k.slide = c.slide * J;
        k.offset = c.offset + j * c.slide;  // in (-slide, J * slide): |offset'| < slide'
        gw_handle* kid = nullptr;
        int rc = gw_create(&k, &kid);
        if (rc) return rc;
        kid->cls_J = J;
        kid->cls_j = j;
        kid->cls_slide = c.slide;
        kid->cls_off = c.offset;
        if (j > 0) {  // one stream for all: the children's launches stay in issue order
            hipStreamSynchronize(kid->stream);
            hipStreamDestroy(kid->stream);
            kid->stream = h->kids[0]->stream;
            kid->shared_stream = true;
        }
        h->kids.push_back(kid);
    }
    h->stream = h->kids[0]->stream;
    h->shared_stream = true;
    return GW_OK;
}

// A first-element handle h (its cfg set): kids[0] the aggregate, kids[1] MIN(sequence);
// minBy / maxBy (GW_FLAG_BY_FIELD): kids[0] alone, MIN / MAX of the field.
static int make_first_element(gw_handle* h) {
    if (h->stream) {  // kernels of its own (sequence, payload log, join) run on kids[0]'s stream
        hipStreamSynchronize(h->stream);
        hipStreamDestroy(h->stream);
        h->stream = nullptr;
    }
    h->fe_by = (h->cfg.flags & GW_FLAG_BY_FIELD) != 0;
    h->fe_by_last = (h->cfg.flags & GW_FLAG_BY_LAST) != 0;
    h->fe_cols = h->fe_by ? 4 : 1;
    gw_config a = h->cfg, b = h->cfg;
    a.flags &= ~(GW_FLAG_FIRST_ELEMENT | GW_FLAG_BY_FIELD | GW_FLAG_BY_LAST);
    b.flags &= ~(GW_FLAG_FIRST_ELEMENT | GW_FLAG_BY_FIELD | GW_FLAG_BY_LAST | GW_FLAG_LATE_SIDE_OUTPUT);
    b.agg = GW_MIN_I64;
    // the sequence operator's values outgrow narrow region records (28 bits) after 2^27
    // records: every record of its first window then went the deferred way (pass 1 ~480 us
    // per 10M-record batch instead of ~70, and a merge) before the handle switched formats at
    // the next window; compact records (32-bit values) from the start
    b.flags |= GW_FLAG_NO_NARROW;
    for (const gw_config* c : {&a, &b}) {
        if (c == &b && h->fe_by) break;
        gw_handle* kid = nullptr;
        const int rc = gw_create(c, &kid);
        if (rc) return rc;
        h->kids.push_back(kid);
    }
    h->fe = true;
    h->stream = h->kids[0]->stream;
    h->shared_stream = true;
    if (hipMalloc((void**)&h->fe_maxts, (size_t)gw_handle::kFeBatches * 8) != hipSuccess ||
        hipMalloc((void**)&h->fe_bad, 4) != hipSuccess) {
        g_create_error = "first-element buffers: out of device memory";
        return GW_E_OOM;
    }
    return GW_OK;
}

int gw_create(const gw_config* cfg, gw_handle** out) {
    if (!cfg || !out) { g_create_error = "null argument"; return GW_E_INVALID; }
    *out = nullptr;
    std::string why;
    int rc = validate(cfg, why);
    if (rc) { g_create_error = why; return rc; }
    gw_handle* h = new (std::nothrow) gw_handle();
    if (!h) { g_create_error = "out of host memory"; return GW_E_OOM; }
    h->cfg = *cfg;
    if (const char* u = getenv("GW_INGEST_UNROLL")) h->ingest_unroll = atoi(u);
    if (const char* u = getenv("GW_REGION_MIN_BATCH")) h->region_min_batch = atoll(u);
    if (const char* u = getenv("GW_BUFFER_RECORDS")) h->buf_limit = std::max<int64_t>(atoll(u), 1);
    h->buf_limit = std::min<int64_t>(h->buf_limit, kMaxIngest);  // buffer offsets stay below 2^32
    if (h->cfg.max_parallelism <= 0) h->cfg.max_parallelism = 128;
    if (h->cfg.parallelism <= 0) h->cfg.parallelism = 1;
    if (h->cfg.max_batch <= 0) h->cfg.max_batch = 1 << 20;
    auto bail = [&](int code, const std::string& msg) {
        g_create_error = msg;
        gw_destroy(h);
        return code;
    };
    hipError_t e = hipSetDevice(cfg->device);
    if (e != hipSuccess) return bail(GW_E_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
    if ((e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess)
        return bail(GW_E_DEVICE, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    if ((e = hipEventCreateWithFlags(&h->ev_in, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&h->ev_out, hipEventDisableTiming)) != hipSuccess)
        return bail(GW_E_DEVICE, std::string("hipEventCreate: ") + hipGetErrorString(e));
    if ((e = hipMalloc((void**)&h->d_st, sizeof(DevStatus))) != hipSuccess ||
        (e = hipMalloc((void**)&h->d_tmp, 64)) != hipSuccess ||
        (e = hipHostMalloc((void**)&h->h_st, sizeof(DevStatus), hipHostMallocDefault)) != hipSuccess)
        return bail(GW_E_DEVICE, std::string("status alloc: ") + hipGetErrorString(e));
    hipMemset(h->d_st, 0, sizeof(DevStatus));
    memset(h->h_st, 0, sizeof(DevStatus));
    for (int i = 0; i < gw_handle::kAsync; ++i) {
        // coherent: the device's stores reach the host without a cache flush on either side
        if ((e = hipHostMalloc((void**)&h->h_st_async[i], sizeof(DevStatus), hipHostMallocCoherent)) != hipSuccess)
            return bail(GW_E_DEVICE, std::string("status alloc: ") + hipGetErrorString(e));
        memset(h->h_st_async[i], 0, sizeof(DevStatus));
    }

    const int agg = cfg->agg;
    const int words = cell_words(agg);
    h->tv.agg = agg;
    h->tv.words = words;
    h->tv.has_mask = !(agg == GW_COUNT || agg == GW_AVG_I64 || agg == GW_AVG_F64);
    int64_t hint = cfg->capacity_hint > 0 ? cfg->capacity_hint : 1 << 16;
    int64_t cap = 1024;
    while ((double)cap * 0.7 < (double)hint) cap *= 2;

    if ((cfg->flags & GW_FLAG_BY_LAST) && !(cfg->flags & GW_FLAG_BY_FIELD))
        return bail(GW_E_INVALID, "GW_FLAG_BY_LAST without GW_FLAG_BY_FIELD");
    if (cfg->assigner == GW_SESSION || cfg->assigner == GW_COUNT_TUMBLING || cfg->assigner == GW_COUNT_SLIDING) {
        if (cfg->flags & (GW_FLAG_FIRST_ELEMENT | GW_FLAG_BY_FIELD))
            return bail(GW_E_UNSUPPORTED, "first-element rows are for tumbling and sliding event-time windows");
        h->session = true;  // the per-key slot path (session merging or count windows)
        rc = session_create(h->sess, *cfg, cap, h->stream, h->d_st, why);
        if (rc) return bail(rc, why);
        hipStreamSynchronize(h->stream);
        *out = h;
        return GW_OK;
    }
    if (cfg->flags & (GW_FLAG_FIRST_ELEMENT | GW_FLAG_BY_FIELD)) {
        if (cfg->trigger != GW_EVENT_TIME_TRIGGER)
            return bail(GW_E_UNSUPPORTED, "first-element rows with PurgingTrigger are not supported");
        const int a = cfg->agg;
        if (a == GW_COUNT || a == GW_AVG_I64 || a == GW_AVG_F64)
            return bail(GW_E_INVALID, "first-element rows are for the positional aggregates sum / min / max");
        if ((cfg->flags & GW_FLAG_BY_FIELD) && !(a == GW_MIN_I64 || a == GW_MAX_I64 || a == GW_MIN_F64 || a == GW_MAX_F64))
            return bail(GW_E_INVALID, "minBy / maxBy (GW_FLAG_BY_FIELD) take GW_MIN_* / GW_MAX_*");
        // the last of equal elements of a lateness re-firing's prefix state would need the
        // re-firing record's sequence per row
        if ((cfg->flags & GW_FLAG_BY_LAST) && cfg->allowed_lateness > 0)
            return bail(GW_E_UNSUPPORTED, "minBy / maxBy with first = false under allowed lateness");
        rc = make_first_element(h);
        if (rc) return bail(rc, g_create_error);
        *out = h;
        return GW_OK;
    }
    const int64_t size = cfg->size;
    const int64_t slide = cfg->assigner == GW_TUMBLING ? cfg->size : cfg->slide;
    pane_geometry(size, slide, h->g, h->n, h->m);
    h->gap_size = size < slide ? size : 0;
    // ring: n panes of the oldest unfired window + at least one pane ahead, filling
    // the slot up to the next 64-byte line
    int64_t need = ring_need(size, slide, cfg->allowed_lateness);
    if (need > kMaxRing) {
        // more panes than one ring holds: split the windows into J classes (k mod J), each a
        // sliding assigner of slide J * slide whose ring fits (gcd(size, J * slide) grows)
        const int64_t J = class_count(size, slide, cfg->allowed_lateness);
        if (J == 0)
            return bail(GW_E_UNSUPPORTED, cfg->allowed_lateness > 0
                                              ? "allowed lateness spanning more than 64 panes of the ring is not "
                                                "supported on the GPU path"
                                              : "no split of the windows into classes fits a ring of 64 panes");
        rc = make_composite(h, J);
        if (rc) return bail(rc, g_create_error);
        *out = h;
        return GW_OK;
    }
    int stride_w = (int)(((2 + need * words) + 7) / 8 * 8);
    int R = (stride_w - 2) / words;
    if (R > kMaxRing) R = kMaxRing;
    h->R = R;
    h->tv.ring = R;
    h->div = make_udiv((uint64_t)h->g);
    h->fired_k = h->k_for_wm(INT64_MIN) + 1;
    h->B = h->fired_k * h->m;
    rc = h->alloc_table(h->tv, std::max<int64_t>(1024, (int64_t)((double)hint / gw_handle::kTableLoad) + 1));
    if (rc) return bail(rc, h->err);
    h->table_bytes = gw_handle::pane_table_bytes(h->tv);
    rc = h->ensure_deferred(1 << 16);
    if (rc) return bail(rc, h->err);
    rc = h->ensure_output(hint);  // one fired window per expected key, before the first fire
    if (rc) return bail(rc, h->err);
    if ((e = hipStreamSynchronize(h->stream)) != hipSuccess)
        return bail(GW_E_DEVICE, std::string("init: ") + hipGetErrorString(e));
    *out = h;
    return GW_OK;
}

int gw_destroy(gw_handle* h) {
    if (!h) return GW_OK;
    if (!h->kids.empty()) {
        for (size_t j = h->kids.size(); j-- > 0;) gw_destroy(h->kids[j]);  // child 0 owns the stream
        h->kids.clear();
        h->stream = nullptr;
        if (h->c_key) { hipFree(h->c_key); hipFree(h->c_start); hipFree(h->c_end); hipFree(h->c_res); }
        if (h->c_pay) hipFree(h->c_pay);
        if (h->fe_log) hipFree(h->fe_log);
        if (h->fe_seqbuf) hipFree(h->fe_seqbuf);
        if (h->fe_maxts) hipFree(h->fe_maxts);
        if (h->fe_bad) hipFree(h->fe_bad);
        if (h->fe_scratch) hipFree(h->fe_scratch);
    }
    h->hp.dump();
    if (h->stream) hipStreamSynchronize(h->stream);
    if (h->pk_stage) hipFree(h->pk_stage);
    h->khm_free();
    if (h->sess) session_destroy(h->sess);
    h->ov_free();
    if (h->tv.base) hipFree(h->tv.base);
    for (int b = 0; b < 2; ++b) {
        if (h->dk[b]) { hipFree(h->dk[b]); hipFree(h->dp[b]); hipFree(h->da0[b]); hipFree(h->da1[b]); }
    }
    if (h->o_key) { hipFree(h->o_key); hipFree(h->o_start); hipFree(h->o_end); hipFree(h->o_res); }
    for (int c = 0; c < 5; ++c)
        if (h->rf[c]) hipFree(h->rf[c]);
    for (int c = 0; c < 3; ++c)
        if (h->lo_buf[c]) hipFree(h->lo_buf[c]);
    if (h->rf_sort) hipFree(h->rf_sort);
    h->free_stage();
    h->free_region();
    if (h->rbeg) hipFree(h->rbeg);
    if (h->d_st) hipFree(h->d_st);
    if (h->d_tmp) hipFree(h->d_tmp);
    if (h->h_st) hipHostFree(h->h_st);
    for (int i = 0; i < gw_handle::kAsync; ++i)
        if (h->h_st_async[i]) hipHostFree(h->h_st_async[i]);
    h->t_ingest.destroy();
    h->t_fire.destroy();
    h->t_apply.destroy();
    if (h->d_chk) hipFree(h->d_chk);
    if (h->nb_scratch) hipFree(h->nb_scratch);
    if (h->nb_cols) hipFree(h->nb_cols);
    if (h->nb_wm) hipFree(h->nb_wm);
    if (h->d_nbst) hipFree(h->d_nbst);
    if (h->h_nbst) hipHostFree(h->h_nbst);
    if (h->h_nbwm) hipHostFree(h->h_nbwm);
    if (h->h_nbbytes) hipHostFree(h->h_nbbytes);
    if (h->d_nbbytes) hipFree(h->d_nbbytes);
    h->free_stage();
    if (h->h_bounce) hipHostFree(h->h_bounce);
    for (auto ev : h->ev_bounce)
        if (ev) hipEventDestroy(ev);
    for (int t = 0; t < gw_handle::kStageBufs; ++t)
        if (h->ev_dread[t]) hipEventDestroy(h->ev_dread[t]);
    if (h->cstream) hipStreamDestroy(h->cstream);
    for (size_t i = 0; i < h->cx.size(); ++i) {
        hipStreamDestroy(h->cx[i]);
        hipEventDestroy(h->cx_ev[i]);
    }
    if (h->ev_fork) hipEventDestroy(h->ev_fork);
    if (h->ev_in) hipEventDestroy(h->ev_in);
    if (h->ev_out) hipEventDestroy(h->ev_out);
    if (h->stream && !h->shared_stream) hipStreamDestroy(h->stream);
    delete h;
    return GW_OK;
}

static int ingest_device_impl(gw_handle* h, int64_t n, const int64_t* key, const int64_t* ts,
                              const int64_t* val) {
    if (h->session) {
        // the grouping sort takes < 2^30 records (gw_sort.h kSortMaxRecords): larger calls go
        // in pieces, each at the same watermark -- the reference processes them one by one
        // anyway, and every piece keeps its records' arrival order
        for (int64_t off = 0; off < n || (n <= 0 && off == 0); off += kSortMaxRecords) {
            const int64_t c = std::min<int64_t>(kSortMaxRecords, n - off);
            int rc = session_ingest(h->sess, c, key + off, ts ? ts + off : nullptr, val ? val + off : nullptr, h->wm,
                                    h->err);
            if (rc != GW_OK) {
                if (rc == GW_E_DEVICE || rc == GW_E_NO_TIMESTAMP || rc == GW_E_RANGE) h->failed = true;
                return rc;
            }
            if (n <= 0) break;
        }
        h->stats.events_in += n;
        h->stats.batches++;
        return GW_OK;
    }
    // the region buffer indexes records with 32-bit offsets: split very large calls
    for (int64_t off = 0; off < n; off += kMaxIngest) {
        const int64_t c = std::min<int64_t>(kMaxIngest, n - off);
        int rc = h->ingest_pane(c, key + off, ts + off, val ? val + off : nullptr);
        if (rc) return rc;
    }
    return GW_OK;
}

// ---- window-class composite: every call goes to each child, results are combined ----
static int kid_rc(gw_handle* h, gw_handle* kid, int rc) {
    return rc == GW_OK ? GW_OK : h->fail(rc, "%s", kid->err.c_str());
}
#define FOR_KIDS(call)                                                                   \
    do {                                                                                 \
        for (gw_handle* k_ : h->kids) {                                                  \
            gw_handle* kid = k_;                                                         \
            const int rc_ = (call);                                                      \
            if (rc_ != GW_OK && rc_ != GW_E_OUTPUT_FULL) return kid_rc(h, kid, rc_);      \
        }                                                                                \
    } while (0)

// ---- first-element handle (GW_FLAG_FIRST_ELEMENT, gw_first.hip) ----------------------
// Row buffers of the joined rows (key, start, end, result, payload) for `need` rows in all.
static int fe_reserve_rows(gw_handle* h, int64_t need) {
    if (need <= h->c_cap) return GW_OK;
    const int64_t cap = std::max<int64_t>(need, 2 * h->c_cap);
    int64_t* nb[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    for (int q = 0; q < 5; ++q) {
        if (hipMalloc((void**)&nb[q], (size_t)cap * 8) != hipSuccess) {
            for (int r = 0; r < q; ++r) hipFree(nb[r]);
            return h->fail(GW_E_OOM, "first-element row buffer: out of device memory");
        }
    }
    int64_t* old[5] = {h->c_key, h->c_start, h->c_end, h->c_res, h->c_pay};
    const int64_t live = h->c_rows - h->c_head;
    for (int q = 0; q < 5; ++q)
        if (old[q] && live) hipMemcpyAsync(nb[q], old[q] + h->c_head, live * 8, hipMemcpyDeviceToDevice, h->stream);
    hipStreamSynchronize(h->stream);
    for (int q = 0; q < 5; ++q)
        if (old[q]) hipFree(old[q]);
    h->c_key = nb[0]; h->c_start = nb[1]; h->c_end = nb[2]; h->c_res = nb[3]; h->c_pay = nb[4];
    h->c_cap = cap;
    h->c_rows = live;
    h->c_head = 0;
    return GW_OK;
}

static int fe_reserve_scratch(gw_handle* h, size_t need) {
    if (need <= h->fe_scratch_bytes) return GW_OK;
    if (h->fe_scratch) {
        hipStreamSynchronize(h->stream);
        hipFree(h->fe_scratch);
    }
    h->fe_scratch = nullptr;
    h->fe_scratch_bytes = 0;
    if (hipMalloc(&h->fe_scratch, need) != hipSuccess) return h->fail(GW_E_OOM, "first-element join scratch");
    h->fe_scratch_bytes = need;
    return GW_OK;
}

// minBy / maxBy: per (key, window start, MIN / MAX) the sequence and payload of the window's
// element (gw_first.hip fe_by_select).  o_seq / o_pay may be null.
static int by_select(gw_handle* h, int64_t n, const int64_t* key, const int64_t* start, const int64_t* res,
                     int64_t* o_seq, int64_t* o_pay) {
    if (n <= 0) return GW_OK;
    int rc = fe_reserve_scratch(h, fe_by_scratch_bytes(n));
    if (rc) return rc;
    const int64_t slide = h->cfg.assigner == GW_TUMBLING ? h->cfg.size : h->cfg.slide;
    const bool f64 = h->cfg.agg == GW_MIN_F64 || h->cfg.agg == GW_MAX_F64;
    hipError_t e = hipMemsetAsync(h->fe_bad, 0, 4, h->stream);
    if (e == hipSuccess)
        e = fe_by_select(n, key, start, res, h->fe_log, h->fe_log_cap, h->fe_log_base, h->fe_seq, h->fe_restored_end,
                         h->cfg.offset, slide, h->cfg.size, h->fe_by_last, f64,
                         h->cfg.agg == GW_MAX_I64 || h->cfg.agg == GW_MAX_F64, o_seq, o_pay, h->fe_scratch,
                         h->fe_scratch_bytes, h->fe_bad, h->stream);
    int32_t bad = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, h->fe_bad, 4, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return h->fail(GW_E_DEVICE, "minBy / maxBy element: %s", hipGetErrorString(e));
    if (bad) return h->fail(GW_E_STATE, "minBy / maxBy element: a window's element is not in the log");
    return GW_OK;
}

// The rows both operators fired, joined by (key, window start) with the payload of the
// window's first element, appended to the c_* rows; then the payloads no window can need
// any more leave the log.  minBy / maxBy: kids[0]'s rows with their element's payload.
static int fe_gather(gw_handle* h) {
    gw_handle* A = h->kids[0];
    int64_t na = 0, nb = 0;
    int rc = gw_pending_rows(A, &na);
    if (rc) return kid_rc(h, A, rc);
    if (h->fe_by) {
        if (na <= 0) return GW_OK;
        const int64_t *ak, *as, *ae;
        const void* ar;
        int64_t x = 0;
        if ((rc = gw_rows_device(A, &ak, &as, &ae, &ar, &x))) return kid_rc(h, A, rc);
        if ((rc = fe_reserve_rows(h, h->c_rows + na))) return rc;
        const int64_t o = h->c_rows;
        const int64_t* src[4] = {ak, as, ae, (const int64_t*)ar};
        int64_t* dst[4] = {h->c_key + o, h->c_start + o, h->c_end + o, h->c_res + o};
        for (int q = 0; q < 4; ++q)
            if (hipMemcpyAsync(dst[q], src[q], (size_t)na * 8, hipMemcpyDeviceToDevice, h->stream) != hipSuccess)
                return h->fail(GW_E_DEVICE, "minBy / maxBy rows");
        if ((rc = by_select(h, na, ak, as, (const int64_t*)ar, nullptr, h->c_pay + o))) return rc;
        h->c_rows += na;
        if ((rc = gw_clear_rows(A))) return kid_rc(h, A, rc);
        return GW_OK;
    }
    gw_handle* B = h->kids[1];
    if ((rc = gw_pending_rows(B, &nb))) return kid_rc(h, B, rc);
    if (na != nb) return h->fail(GW_E_STATE, "first-element rows out of step (%lld vs %lld)", (long long)na, (long long)nb);
    if (na > 0) {
        const int64_t *ak, *as, *ae, *bk, *bs, *be;
        const void *ar, *br;
        int64_t x = 0;
        if ((rc = gw_rows_device(A, &ak, &as, &ae, &ar, &x))) return kid_rc(h, A, rc);
        if ((rc = gw_rows_device(B, &bk, &bs, &be, &br, &x))) return kid_rc(h, B, rc);
        if (B->stream != h->stream) {
            // B (e.g. a window-class composite) gathers its rows on its own stream: the join
            // on h's stream reads them only after those copies
            if (hipEventRecord(h->ev_out, B->stream) != hipSuccess || hipStreamWaitEvent(h->stream, h->ev_out, 0) != hipSuccess)
                return h->fail(GW_E_DEVICE, "first-element join: stream ordering");
        }
        if ((rc = fe_reserve_rows(h, h->c_rows + na))) return rc;
        if ((rc = fe_reserve_scratch(h, fe_join_scratch_bytes(na)))) return rc;
        const int64_t o = h->c_rows;
        hipError_t e = hipMemsetAsync(h->fe_bad, 0, 4, h->stream);
        if (e == hipSuccess)
            e = fe_join(na, ak, as, ae, (const int64_t*)ar, bk, bs, (const int64_t*)br, h->fe_log, h->fe_log_base,
                        h->fe_log_cap, h->c_key + o, h->c_start + o, h->c_end + o, h->c_res + o, h->c_pay + o,
                        h->fe_scratch, h->fe_scratch_bytes, h->fe_bad, h->stream);
        int32_t bad = 0;
        if (e == hipSuccess) e = hipMemcpyAsync(&bad, h->fe_bad, 4, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return h->fail(GW_E_DEVICE, "first-element join: %s", hipGetErrorString(e));
        if (bad) return h->fail(GW_E_STATE, "first-element join: %s", bad & 1 ? "rows differ" : "payload released");
        h->c_rows += na;
        if ((rc = gw_clear_rows(A))) return kid_rc(h, A, rc);
        if ((rc = gw_clear_rows(B))) return kid_rc(h, B, rc);
    }
    return GW_OK;
}

// Release the payloads no window can need any more: a batch whose largest timestamp's
// windows are all cleaned (maxTs + size - 1 + lateness <= wm: WindowOperator.cleanupTime).
// Runs after a fire (cleanup happens then) and when the log would have to grow, so a
// watermark that fires nothing costs no host synchronisation.
static int fe_release(gw_handle* h) {
    const int64_t wm = h->fe_wm;
    if (!h->fe_batches.empty()) {
        bool any = false;  // each batch's max timestamp crosses to the host once
        for (auto& b : h->fe_batches) {
            if (b.known) continue;
            if (hipMemcpyAsync(&b.max_ts, h->fe_maxts + b.slot, 8, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
                return h->fail(GW_E_DEVICE, "first-element log");
            b.known = any = true;
        }
        if (any && hipStreamSynchronize(h->stream) != hipSuccess) return h->fail(GW_E_DEVICE, "first-element log");
        size_t q = 0;
        for (; q < h->fe_batches.size(); ++q) {
            const int64_t mx = h->fe_batches[q].max_ts;
            const i128 ct = (i128)mx + (i128)h->cfg.size - 1 + (i128)h->cfg.allowed_lateness;
            if (mx != INT64_MIN && ct > (i128)wm) break;
            h->fe_log_base = h->fe_batches[q].seq_end;
        }
        h->fe_batches.erase(h->fe_batches.begin(), h->fe_batches.begin() + q);
        // a long lateness keeps many batches: merge neighbours (the later end, the larger
        // max timestamp -- released no earlier than either) so the list stays short
        if (h->fe_batches.size() > 1024) {
            std::vector<gw_handle::FeBatch> m;
            for (size_t i = 0; i < h->fe_batches.size(); i += 2) {
                gw_handle::FeBatch b = h->fe_batches[i];
                if (i + 1 < h->fe_batches.size()) {
                    b.seq_end = h->fe_batches[i + 1].seq_end;
                    b.max_ts = std::max(b.max_ts, h->fe_batches[i + 1].max_ts);
                }
                m.push_back(b);
            }
            h->fe_batches.swap(m);
        }
    }
    return GW_OK;
}

// Room in the payload log (a ring of the live sequences [fe_log_base, fe_seq + n)) for n
// more sequences: release what no window needs any more, then grow.
static int fe_log_reserve(gw_handle* h, int64_t n) {
    hipStream_t s = h->stream;
    if (h->fe_seq + n - h->fe_log_base > h->fe_log_cap || (int64_t)h->fe_batches.size() >= gw_handle::kFeBatches - 1) {
        const int rc = fe_release(h);
        if (rc) return rc;
    }
    const int64_t need = h->fe_seq + n - h->fe_log_base;
    if (need > h->fe_log_cap) {
        const int64_t ncap = std::max<int64_t>(2 * need, 1 << 20);
        int64_t* nl = nullptr;
        if (hipMalloc((void**)&nl, (size_t)ncap * 8 * h->fe_cols) != hipSuccess) return h->fail(GW_E_OOM, "payload log");
        hipError_t e = hipSuccess;
        for (int c = 0; c < h->fe_cols && h->fe_log && e == hipSuccess; ++c)  // column c at c * cap
            e = fe_log_regrow(h->fe_log + c * h->fe_log_cap, h->fe_log_cap, nl + c * ncap, ncap, h->fe_log_base,
                              h->fe_seq, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (h->fe_log) hipFree(h->fe_log);
        h->fe_log = nl;
        h->fe_log_cap = ncap;
        if (e != hipSuccess) return h->fail(GW_E_DEVICE, "payload log: %s", hipGetErrorString(e));
    }
    return GW_OK;
}

int gw_ingest_payload_device(gw_handle* h, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                             const int64_t* d_ts, const void* d_value, const int64_t* d_payload, void* stream) {
    if (!h) return GW_E_INVALID;
    if (!h->fe) return h->fail(GW_E_INVALID, "gw_ingest_payload*: not a GW_FLAG_FIRST_ELEMENT handle");
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    if (n < 0 || (n > 0 && (!d_key || !d_ts || !d_value || !d_payload)))
        return h->fail(GW_E_INVALID, "null key/ts/value/payload column");
    hipSetDevice(h->cfg.device);
    hipStream_t s = h->stream, ps = (hipStream_t)stream;
    if (ps != s) {
        hipEventRecord(h->ev_in, ps);
        hipStreamWaitEvent(s, h->ev_in, 0);
    }
    if (n == 0) return GW_OK;
    // arrival sequence of the batch's records (kids[1] folds its minimum per window)
    if (n > h->fe_seqbuf_cap) {
        hipStreamSynchronize(s);
        if (h->fe_seqbuf) hipFree(h->fe_seqbuf);
        h->fe_seqbuf = nullptr;
        h->fe_seqbuf_cap = 0;
        if (hipMalloc((void**)&h->fe_seqbuf, (size_t)n * 8) != hipSuccess) return h->fail(GW_E_OOM, "sequence buffer");
        h->fe_seqbuf_cap = n;
    }
    hipError_t e = h->fe_by ? hipSuccess : fe_iota64(h->fe_seqbuf, n, h->fe_seq, s);
    if (e == hipSuccess) {
        const int rc = fe_log_reserve(h, n);
        if (rc) return rc;
        e = fe_log_append(h->fe_log, h->fe_log_cap, h->fe_seq, d_payload, n, s);
        if (h->fe_by) {  // minBy / maxBy: key, ts and field beside the payload
            const int64_t* col[3] = {d_key, d_ts, (const int64_t*)d_value};
            for (int c = 0; c < 3 && e == hipSuccess; ++c)
                e = fe_log_append(h->fe_log + (c + 1) * h->fe_log_cap, h->fe_log_cap, h->fe_seq, col[c], n, s);
        }
    }
    if ((int64_t)h->fe_batches.size() >= gw_handle::kFeBatches - 1)
        return h->fail(GW_E_STATE, "first-element log: too many batches without a watermark");
    const int64_t slot = h->fe_batch_no % gw_handle::kFeBatches;
    if (e == hipSuccess) e = fe_iota64(h->fe_maxts + slot, 1, INT64_MIN, s);
    if (e == hipSuccess) e = fe_max_ts(d_ts, n, h->fe_maxts + slot, s);
    if (e != hipSuccess) return h->fail(GW_E_DEVICE, "first-element ingest: %s", hipGetErrorString(e));
    h->fe_batches.push_back({h->fe_seq + n, slot, INT64_MIN, false});
    h->fe_batch_no++;
    int rc = gw_ingest_device(h->kids[0], n, d_key, d_key_hash, d_ts, d_value, (void*)s);
    if (rc) return kid_rc(h, h->kids[0], rc);
    if (!h->fe_by && (rc = gw_ingest_device(h->kids[1], n, d_key, d_key_hash, d_ts, h->fe_seqbuf, (void*)s)))
        return kid_rc(h, h->kids[1], rc);
    h->fe_seq += n;
    if (ps != s) {
        hipEventRecord(h->ev_out, s);
        hipStreamWaitEvent(ps, h->ev_out, 0);
    }
    return GW_OK;
}

int gw_ingest_payload(gw_handle* h, int64_t n, const int64_t* key, const int32_t* key_hash, const int64_t* ts,
                      const void* value, const int64_t* payload) {
    if (!h) return GW_E_INVALID;
    if (!h->fe) return h->fail(GW_E_INVALID, "gw_ingest_payload*: not a GW_FLAG_FIRST_ELEMENT handle");
    if (n < 0 || (n > 0 && (!key || !ts || !value || !payload)))
        return h->fail(GW_E_INVALID, "null key/ts/value/payload column");
    if (n == 0) return GW_OK;
    hipSetDevice(h->cfg.device);
    // host columns: one device copy of each (synchronous), then the device path
    int64_t* d = nullptr;
    int32_t* dh = nullptr;
    if (hipMalloc((void**)&d, (size_t)n * 32) != hipSuccess) return h->fail(GW_E_OOM, "payload staging");
    if (key_hash && hipMalloc((void**)&dh, (size_t)n * 4) != hipSuccess) {
        hipFree(d);
        return h->fail(GW_E_OOM, "payload staging");
    }
    hipError_t e = hipMemcpyAsync(d, key, n * 8, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d + n, ts, n * 8, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d + 2 * n, value, n * 8, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d + 3 * n, payload, n * 8, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess && dh) e = hipMemcpyAsync(dh, key_hash, n * 4, hipMemcpyHostToDevice, h->stream);
    int rc = e == hipSuccess ? gw_ingest_payload_device(h, n, d, dh, d + n, d + 2 * n, d + 3 * n, h->stream)
                             : h->fail(GW_E_DEVICE, "H2D: %s", hipGetErrorString(e));
    hipStreamSynchronize(h->stream);
    hipFree(d);
    if (dh) hipFree(dh);
    return rc;
}

int gw_drain_payload(gw_handle* h, int64_t* key, int64_t* start, int64_t* end, void* result, int64_t* payload,
                     int64_t cap, int64_t* n) {
    if (!h || !n) return GW_E_INVALID;
    *n = 0;
    if (!h->fe) return h->fail(GW_E_INVALID, "gw_drain_payload: not a GW_FLAG_FIRST_ELEMENT handle");
    const int64_t c = std::min(cap, h->c_rows - h->c_head);
    if (c > 0) {
        const int64_t o = h->c_head;
        int64_t* dst[5] = {key, start, end, (int64_t*)result, payload};
        int64_t* src[5] = {h->c_key, h->c_start, h->c_end, h->c_res, h->c_pay};
        hipError_t e = hipSuccess;
        for (int q = 0; q < 5 && e == hipSuccess; ++q)
            if (dst[q]) e = hipMemcpyAsync(dst[q], src[q] + o, c * 8, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return h->fail(GW_E_DEVICE, "D2H rows: %s", hipGetErrorString(e));
        h->c_head += c;
        if (h->c_head == h->c_rows) h->c_head = h->c_rows = 0;
    }
    *n = c;
    return h->c_rows - h->c_head > 0 ? GW_E_OUTPUT_FULL : GW_OK;
}

static int stage_ingest(gw_handle* h, int slot, int64_t n, bool with_hash, bool with_value);

int gw_ingest(gw_handle* h, int64_t n, const int64_t* key, const int32_t* key_hash, const int64_t* ts,
              const void* value) {
    if (!h) return GW_E_INVALID;
    if (h->fe) return h->fail(GW_E_INVALID, "GW_FLAG_FIRST_ELEMENT handle: records need their payload (gw_ingest_payload)");
    if (!h->kids.empty()) {
        FOR_KIDS(gw_ingest(kid, n, key, key_hash, ts, value));
        return GW_OK;
    }
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    if (n < 0 || (n > 0 && (!key || !ts))) return h->fail(GW_E_INVALID, "null key/ts column");
    if (n > 0 && !value && h->cfg.agg != GW_COUNT) return h->fail(GW_E_INVALID, "value column required");
    if (h->slots_out && n > 0)  // gw_ingest copies through the same pinned slots the caller now fills
        return h->fail(GW_E_STATE, "gw_ingest on a handle whose pinned slots were handed out (gw_stage_columns): "
                                   "ingest them with gw_ingest_stage");
    hipSetDevice(h->cfg.device);
    const int64_t chunk = h->cfg.max_batch;
    for (int64_t off = 0; off < n; off += chunk) {
        const int64_t c = std::min(chunk, n - off);
        int rc = h->ensure_stage(c);
        if (rc) return rc;
        const int slot = h->stage_next;
        h->stage_next ^= 1;
        if ((rc = h->slot_ready(slot))) return rc;
        int64_t* hs = h->h_slot[slot];
        const int64_t cap = h->slot_cap;
        par_memcpy(hs, key + off, (size_t)c * 8);
        par_memcpy(hs + cap, ts + off, (size_t)c * 8);
        if (value) par_memcpy(hs + 2 * cap, (const int64_t*)value + off, (size_t)c * 8);
        if (key_hash) memcpy(hs + 3 * cap, key_hash + off, (size_t)c * 4);
        if ((rc = stage_ingest(h, slot, c, key_hash != nullptr, value != nullptr))) return rc;
    }
    return GW_OK;
}

// One filled pinned slot -> the next device staging buffer, on the copy stream (after the
// ingest that last read that buffer).  cols: GW_STAGE_VALUE | GW_STAGE_KEY_HASH.
static int stage_send(gw_handle* h, int slot, int64_t n, int cols) {
    const int t = h->send_turn;
    if (h->pre_valid[t]) return h->fail(GW_E_STATE, "staging: every device buffer holds a batch not yet ingested");
    const int64_t cap = h->slot_cap;
    int64_t* hs = h->h_slot[slot];
    int64_t* ds = h->d_stage2[t];
    hipError_t e = hipSuccess;
    if (h->dread_valid[t]) e = hipStreamWaitEvent(h->cstream, h->ev_dread[t], 0);
    // the columns (key, ts, value, key hash), each cut into one piece per copy stream
    const int ns = h->cx.empty() ? 1 : (int)h->cx.size();
    if (ns > 1 && e == hipSuccess) {
        e = hipEventRecord(h->ev_fork, h->cstream);
        for (int k = 0; k < ns && e == hipSuccess; ++k) e = hipStreamWaitEvent(h->cx[k], h->ev_fork, 0);
    }
    const int64_t piece = (n + ns - 1) / ns;
    for (int c = 0; c < 4 && e == hipSuccess; ++c) {
        if (c == 2 && !(cols & GW_STAGE_VALUE)) continue;
        if (c == 3 && !(cols & GW_STAGE_KEY_HASH)) continue;
        const size_t w = c == 3 ? 4 : 8;
        char* d = reinterpret_cast<char*>(ds + c * cap);
        const char* hsrc = reinterpret_cast<const char*>(hs + c * cap);
        for (int k = 0; k < ns && e == hipSuccess; ++k) {
            const int64_t lo = k * piece, hi = std::min(n, lo + piece);
            if (hi > lo)
                e = hipMemcpyAsync(d + lo * w, hsrc + lo * w, (size_t)(hi - lo) * w, hipMemcpyHostToDevice,
                                   ns > 1 ? h->cx[k] : h->cstream);
        }
    }
    if (ns > 1)
        for (int k = 0; k < ns && e == hipSuccess; ++k) {
            e = hipEventRecord(h->cx_ev[k], h->cx[k]);
            if (e == hipSuccess) e = hipStreamWaitEvent(h->cstream, h->cx_ev[k], 0);
        }
    if (e == hipSuccess) e = hipEventRecord(h->ev_slot[slot], h->cstream);
    if (e != hipSuccess) return h->fail(GW_E_DEVICE, "H2D: %s", hipGetErrorString(e));
    h->slot_used[slot] = true;
    h->pre_valid[t] = true;
    h->pre_slot[t] = slot;
    h->pre_n[t] = n;
    h->pre_cols[t] = cols;
    h->send_turn = (h->send_turn + 1) % gw_handle::kStageBufs;
    return GW_OK;
}

// A staged batch -> ingest (the handle's stream): the slot sent ahead, or sent now.
static int stage_ingest(gw_handle* h, int slot, int64_t n, bool with_hash, bool with_value) {
    const int cols = (with_value ? GW_STAGE_VALUE : 0) | (with_hash ? GW_STAGE_KEY_HASH : 0);
    const int t = h->dturn;
    int rc;
    if (!h->pre_valid[t]) {
        if (h->send_turn != t)  // a later batch went ahead of this one
            return h->fail(GW_E_STATE, "staging: ingest of slot %d, which was not sent, after later batches were", slot);
        if ((rc = stage_send(h, slot, n, cols))) return rc;
    } else if (h->pre_slot[t] != slot || h->pre_n[t] != n || h->pre_cols[t] != cols) {
        return h->fail(GW_E_STATE, "staging: ingest of slot %d (%lld records) while slot %d (%lld) was sent first",
                       slot, (long long)n, h->pre_slot[t], (long long)h->pre_n[t]);
    }
    h->pre_valid[t] = false;
    h->dturn = (h->dturn + 1) % gw_handle::kStageBufs;
    const int64_t cap = h->slot_cap;
    int64_t* ds = h->d_stage2[t];
    int32_t* dh = (int32_t*)(ds + 3 * cap);
    if (hipStreamWaitEvent(h->stream, h->ev_slot[slot], 0) != hipSuccess) return h->fail(GW_E_DEVICE, "staging event");
    rc = h->check_keys(n, ds, with_hash ? dh : nullptr);
    if (rc == GW_OK) rc = ingest_device_impl(h, n, ds, ds + cap, with_value ? ds + 2 * cap : nullptr);
    if (hipEventRecord(h->ev_dread[t], h->stream) != hipSuccess) return h->fail(GW_E_DEVICE, "staging event");
    h->dread_valid[t] = true;
    return rc;
}

int gw_stage_alloc(gw_handle* h, int32_t slots, int64_t cap) {
    if (!h || slots < 1 || slots > 4096 || cap < 1) return GW_E_INVALID;
    if (!h->kids.empty() || h->fe) return h->fail(GW_E_UNSUPPORTED, "staged ingest on a composite / first-element handle");
    hipSetDevice(h->cfg.device);
    return h->ensure_stage(cap, slots);
}

int gw_stage_columns(gw_handle* h, int32_t slot, int64_t** key, int32_t** key_hash, int64_t** ts, int64_t** value) {
    if (!h || slot < 0 || slot >= (int)h->h_slot.size()) return GW_E_INVALID;
    hipSetDevice(h->cfg.device);
    const int rc = h->slot_ready(slot);
    if (rc) return rc;
    int64_t* hs = h->h_slot[slot];
    h->slots_out = true;
    if (key) *key = hs;
    if (ts) *ts = hs + h->slot_cap;
    if (value) *value = hs + 2 * h->slot_cap;
    if (key_hash) *key_hash = (int32_t*)(hs + 3 * h->slot_cap);
    return GW_OK;
}

int gw_stage_send(gw_handle* h, int32_t slot, int64_t n, int32_t cols) {
    if (!h || slot < 0 || slot >= (int)h->h_slot.size() || n < 0 || n > h->slot_cap) return GW_E_INVALID;
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    if (n > 0 && !(cols & GW_STAGE_VALUE) && h->cfg.agg != GW_COUNT) return h->fail(GW_E_INVALID, "value column required");
    hipSetDevice(h->cfg.device);
    if (n == 0) return GW_OK;
    return stage_send(h, slot, n, cols & (GW_STAGE_VALUE | GW_STAGE_KEY_HASH));
}

int gw_ingest_stage(gw_handle* h, int32_t slot, int64_t n, int32_t cols) {
    if (!h || slot < 0 || slot >= (int)h->h_slot.size() || n < 0 || n > h->slot_cap) return GW_E_INVALID;
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    const bool with_value = (cols & GW_STAGE_VALUE) != 0, with_hash = (cols & GW_STAGE_KEY_HASH) != 0;
    if (n > 0 && !with_value && h->cfg.agg != GW_COUNT) return h->fail(GW_E_INVALID, "value column required");
    hipSetDevice(h->cfg.device);
    if (n == 0) return GW_OK;
    return stage_ingest(h, slot, n, with_hash, with_value);
}

int gw_ingest_device(gw_handle* h, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                     const int64_t* d_ts, const void* d_value, void* stream) {
    if (!h) return GW_E_INVALID;
    if (h->fe)
        return h->fail(GW_E_INVALID, "GW_FLAG_FIRST_ELEMENT handle: records need their payload (gw_ingest_payload_device)");
    if (!h->kids.empty()) {  // the children share one stream: order after the producer once
        FOR_KIDS(gw_ingest_device(kid, n, d_key, d_key_hash, d_ts, d_value, stream));
        return GW_OK;
    }
    h->hp.mark();
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    if (n < 0 || (n > 0 && (!d_key || !d_ts))) return h->fail(GW_E_INVALID, "null key/ts column");
    if (n > 0 && !d_value && h->cfg.agg != GW_COUNT) return h->fail(GW_E_INVALID, "value column required");
    hipSetDevice(h->cfg.device);
    // The producer stream (NULL = the default stream) wrote the columns; the handle's
    // non-blocking stream reads them.  Order both ways: the reads after the writes, and
    // whatever the producer stream does next (reusing or freeing the columns) after the
    // reads, so a caching allocator on the producer side needs nothing more.
    hipStream_t ps = (hipStream_t)stream;
    const bool foreign = ps != h->stream;
    if (foreign) {
        hipEventRecord(h->ev_in, ps);
        hipStreamWaitEvent(h->stream, h->ev_in, 0);
    }
    if (n == 0) return GW_OK;
    h->hp.lap(5);
    int rc = h->check_keys(h->pk_w ? h->pk_from : n, d_key, d_key_hash);  // (packed words: routed already)
    if (rc == GW_OK) rc = ingest_device_impl(h, n, d_key, d_ts, (const int64_t*)d_value);
    if (foreign) {
        hipEventRecord(h->ev_out, h->stream);
        hipStreamWaitEvent(ps, h->ev_out, 0);
    }
    return rc;
}

int gw_ingest_packed_device(gw_handle* h, int64_t n_other, const int64_t* d_key, const int64_t* d_ts,
                            const int64_t* d_value, int64_t n_words, const uint64_t* d_words, const gw_pack_geom* g,
                            void* stream) {
    if (!h) return GW_E_INVALID;
    if (n_other < 0 || n_words < 0 || (n_words > 0 && (!d_words || !g || !g->enabled || g->pane <= 0)))
        return h->fail(GW_E_INVALID, "gw_ingest_packed_device: bad word arguments");
    if (n_words == 0) return gw_ingest_device(h, n_other, d_key, nullptr, d_ts, d_value, stream);
    {  // a word's timestamp is its pane's start: only handles whose every decision depends on the
       // pane alone may take it (gpuwin.h gw_pack_geom)
        const gw_config& c = h->cfg;
        const bool fp_in = c.agg == GW_SUM_F64 || c.agg == GW_MIN_F64 || c.agg == GW_MAX_F64 || c.agg == GW_AVG_F64;
        // (window-class composites may: every class window's bounds lie on the pane grid, so a
        // record and its pane's start fall into the same windows of every class)
        if (h->session || h->fe || (c.flags & GW_FLAG_LATE_SIDE_OUTPUT) || fp_in ||
            (c.assigner != GW_TUMBLING && c.assigner != GW_SLIDING))
            return h->fail(GW_E_UNSUPPORTED,
                           "gw_ingest_packed_device: packed words need a plain tumbling / sliding handle over an "
                           "integer aggregate without the late side output (unpack them for this handle)");
        const int64_t size = c.size, slide = c.assigner == GW_TUMBLING ? c.size : c.slide;
        const i128 doff = (i128)c.offset - (i128)g->offset;
        if (size < slide || size % g->pane || slide % g->pane || doff % g->pane)
            return h->fail(GW_E_UNSUPPORTED,
                           "gw_ingest_packed_device: the words' pane geometry (pane %lld, offset %lld) does not "
                           "divide this handle's windows (size %lld, slide %lld, offset %lld)",
                           (long long)g->pane, (long long)g->offset, (long long)size, (long long)slide,
                           (long long)c.offset);
    }
    const bool vals = h->cfg.agg != GW_COUNT;
    if (n_other > 0 && (!d_key || !d_ts || (vals && !d_value))) return h->fail(GW_E_INVALID, "null key/ts/value column");
    const int64_t n = n_other + n_words;
    // columns of no records: any non-null pointer (never read below pk_from = 0)
    const int64_t* dummy = (const int64_t*)d_words;
    const int64_t* k = n_other ? d_key : dummy;
    const int64_t* t = n_other ? d_ts : dummy;
    const int64_t* v = vals ? (n_other ? d_value : dummy) : nullptr;
    const bool plain = !h->fe && h->kids.empty() && !h->session && n <= kMaxIngest;
    if (!plain) {  // unpack into the handle's staging columns on the producer stream, then as usual
        if (n > h->pk_stage_cap) {
            hipStreamSynchronize((hipStream_t)stream);
            hipStreamSynchronize(h->stream);
            hipFree(h->pk_stage);
            h->pk_stage = nullptr;
            const int64_t c = std::max<int64_t>(n + n / 4, 1 << 16);
            if (hipMalloc((void**)&h->pk_stage, (size_t)c * 3 * 8) != hipSuccess)
                return h->fail(GW_E_OOM, "packed staging: out of device memory");
            h->pk_stage_cap = c;
        }
        int64_t* sk = h->pk_stage;
        int64_t* st = sk + h->pk_stage_cap;
        int64_t* sv = vals ? st + h->pk_stage_cap : nullptr;
        hipStream_t ps = (hipStream_t)stream;
        if (n_other > 0) {
            hipMemcpyAsync(sk, d_key, (size_t)n_other * 8, hipMemcpyDeviceToDevice, ps);
            hipMemcpyAsync(st, d_ts, (size_t)n_other * 8, hipMemcpyDeviceToDevice, ps);
            if (sv) hipMemcpyAsync(sv, d_value, (size_t)n_other * 8, hipMemcpyDeviceToDevice, ps);
        }
        if (launch_unpack(n_words, d_words, *g, sk + n_other, st + n_other, sv ? sv + n_other : nullptr, ps) !=
            hipSuccess)
            return h->fail(GW_E_DEVICE, "packed staging: unpack launch failed");
        return gw_ingest_device(h, n, sk, nullptr, st, sv, stream);
    }
    h->pk_w = d_words;
    h->pk_from = n_other;
    h->pk_g = *g;
    const int rc = gw_ingest_device(h, n, k, nullptr, t, v, stream);
    h->pk_w = nullptr;
    h->pk_from = 0;
    return rc;
}

// ---- network-buffer ingest ---------------------------------------------------
// Validates the record layout (and, with agg >= 0, that the aggregated field's type
// suits the aggregate: a Long/Integer/Short/Byte field for the integer aggregates, a
// Double/Float field for the floating-point ones, as SumAggregator / ComparableAggregator
// require a field of the result's type, RS/api/functions/aggregation/SumFunction.java).
static int nb_layout(const gw_record_layout* lay, int agg, NbLayout& L, std::string& why) {
    if (!lay) { why = "null record layout"; return GW_E_INVALID; }
    if (lay->nfields < 1 || lay->nfields > GW_MAX_FIELDS) { why = "layout: 1..8 fields"; return GW_E_INVALID; }
    int off[GW_MAX_FIELDS], vb = 0;
    for (int i = 0; i < lay->nfields; ++i) {
        const int w = nb_field_width(lay->types[i]);
        if (w < 0) { why = std::string("layout: unknown type code '") + lay->types[i] + "'"; return GW_E_INVALID; }
        off[i] = vb;
        vb += w;
    }
    if (lay->key_field < 0 || lay->key_field >= lay->nfields || lay->types[lay->key_field] != 'J') {
        why = "layout: the key field must be a Long ('J')";
        return GW_E_INVALID;
    }
    if (lay->value_field < -1 || lay->value_field >= lay->nfields) { why = "layout: bad value field"; return GW_E_INVALID; }
    L.vbytes = vb;
    L.key_off = off[lay->key_field];
    L.val_off = lay->value_field >= 0 ? off[lay->value_field] : 0;
    L.val_type = lay->value_field >= 0 ? lay->types[lay->value_field] : 0;
    if (agg < 0) return GW_OK;
    if (agg == GW_COUNT) { L.val_type = 0; return GW_OK; }
    if (!L.val_type) { why = "layout: the aggregate needs a value field"; return GW_E_INVALID; }
    const char t = (char)L.val_type;
    const bool fp = result_is_double(agg) && agg != GW_AVG_I64;
    const bool ok = fp ? (t == 'D' || t == 'F') : (t == 'J' || t == 'I' || t == 'S' || t == 'B');
    if (!ok) { why = std::string("layout: field type '") + t + "' does not match the aggregate"; return GW_E_INVALID; }
    return GW_OK;
}

static int nb_status_code(const NbStatus& st, std::string& why) {
#ifdef GW_DEBUG_LOG  // experiment builds only
    fprintf(stderr, "gw netbuf: fallback %llu walkback %llu\n", st.fallback, st.walkback);
#endif
    if (st.corrupt) { why = "Corrupt stream: unknown tag or element length (StreamElementSerializer)"; return GW_E_INVALID; }
    if (st.unsupported) { why = "stream element longer than GW_MAX_ELEMENT bytes"; return GW_E_UNSUPPORTED; }
    if (st.full) { why = "decoded records / watermarks exceed the output capacity"; return GW_E_OUTPUT_FULL; }
    return GW_OK;
}

int gw_decode_serialized(const void* d_bytes, int64_t nbytes, const gw_record_layout* layout, int64_t* d_key,
                         int64_t* d_ts, int64_t* d_value, int64_t rec_cap, int64_t* d_wm_pos, int64_t* d_wm_val,
                         int64_t wm_cap, gw_decode_result* out, void* stream) {
    NbLayout L{};
    std::string why;
    int rc = nb_layout(layout, -1, L, why);
    if (rc) { g_create_error = why; return rc; }
    if (nbytes < 0 || (nbytes > 0 && !d_bytes) || !out || ((uintptr_t)d_bytes & 3)) {
        g_create_error = "bad byte buffer (device pointer, 4-byte aligned)";
        return GW_E_INVALID;
    }
    if ((rec_cap > 0 && (!d_key || !d_ts)) || (wm_cap > 0 && (!d_wm_pos || !d_wm_val))) {
        g_create_error = "null output column";
        return GW_E_INVALID;
    }
    hipStream_t s = (hipStream_t)stream;
    void* scratch = nullptr;
    NbStatus* d_st = nullptr;
    NbStatus hst{};
    hipError_t e = hipMalloc(&scratch, (size_t)nb_scratch_bytes(nbytes));
    if (e == hipSuccess) e = hipMalloc((void**)&d_st, sizeof(NbStatus));
    if (e == hipSuccess)
        e = launch_nb_decode((const uint8_t*)d_bytes, nbytes, L, d_key, d_ts, d_value, rec_cap, d_wm_pos, d_wm_val,
                             wm_cap, scratch, d_st, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&hst, d_st, sizeof(NbStatus), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (scratch) hipFree(scratch);
    if (d_st) hipFree(d_st);
    if (e != hipSuccess) { g_create_error = std::string("decode: ") + hipGetErrorString(e); return GW_E_DEVICE; }
    out->records = hst.records;
    out->watermarks = hst.watermarks;
    out->consumed = hst.consumed;
    out->skipped = (int64_t)hst.skipped;
    rc = nb_status_code(hst, why);
    if (rc) g_create_error = why;
    return rc;
}

static int nb_ensure(gw_handle* h, int64_t nbytes, const NbLayout& L) {
    auto grow = [&](void** p, int64_t& cap, int64_t want, int64_t unit) -> hipError_t {
        if (want <= cap) return hipSuccess;
        if (*p) hipFree(*p);
        *p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(p, (size_t)(want * unit));
        if (e == hipSuccess) cap = want;
        return e;
    };
    const int64_t want = std::max<int64_t>(nbytes, 1 << 16);
    // upper bounds: every element a record without timestamp / a watermark
    const int64_t recs = want / (4 + 1 + L.vbytes) + 1, wms = want / 13 + 1;
    hipError_t e = grow(&h->nb_scratch, h->nb_scratch_cap, nb_scratch_bytes(want), 1);
    if (e == hipSuccess) e = grow((void**)&h->nb_cols, h->nb_rec_cap, recs, 24);
    if (e == hipSuccess) e = grow((void**)&h->nb_wm, h->nb_wm_cap, wms, 16);
    if (e == hipSuccess && !h->d_nbst) e = hipMalloc((void**)&h->d_nbst, sizeof(NbStatus));
    if (e == hipSuccess && !h->h_nbst) e = hipHostMalloc((void**)&h->h_nbst, sizeof(NbStatus), hipHostMallocDefault);
    if (e == hipSuccess && !h->h_nbwm)
        e = hipHostMalloc((void**)&h->h_nbwm, 2 * gw_handle::kNbWmHost * 8, hipHostMallocDefault);
    if (e != hipSuccess) return h->fail(GW_E_OOM, "network-buffer scratch: %s", hipGetErrorString(e));
    return GW_OK;
}

// Decode on the handle's stream, then replay the channel: records between two watermarks
// as one batch, each watermark as gw_advance_watermark (StreamTaskNetworkInput.processElement,
// RS/runtime/io/AbstractStreamTaskNetworkInput.java:210-235; one channel's
// StatusWatermarkValve forwards every advancing watermark, StatusWatermarkValve.java:153-185).
static int nb_ingest_on_stream(gw_handle* h, const uint8_t* d_bytes, int64_t nbytes, const NbLayout& L,
                               int64_t* consumed, int64_t* rows_fired) {
    int rc = nb_ensure(h, nbytes, L);
    if (rc) return rc;
    int64_t* k = h->nb_cols;
    int64_t* t = h->nb_cols + h->nb_rec_cap;
    int64_t* v = h->nb_cols + 2 * h->nb_rec_cap;
    int64_t* wp = h->nb_wm;
    int64_t* wv = h->nb_wm + h->nb_wm_cap;
    hipError_t e = launch_nb_decode(d_bytes, nbytes, L, k, t, L.val_type ? v : nullptr, h->nb_rec_cap, wp, wv,
                                    h->nb_wm_cap, h->nb_scratch, h->d_nbst, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h->h_nbst, h->d_nbst, sizeof(NbStatus), hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h->h_nbwm, wp, gw_handle::kNbWmHost * 8, hipMemcpyDeviceToHost, h->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(h->h_nbwm + gw_handle::kNbWmHost, wv, gw_handle::kNbWmHost * 8, hipMemcpyDeviceToHost,
                           h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return h->fail(GW_E_DEVICE, "network-buffer decode: %s", hipGetErrorString(e));
    const NbStatus st = *h->h_nbst;
    std::string why;
    rc = nb_status_code(st, why);
    if (rc) {
        h->fail(rc, "%s", why.c_str());
        if (rc == GW_E_INVALID) h->failed = true;  // IOException: the task fails
        return rc;
    }
    std::vector<int64_t> wpos, wval;
    const int64_t nw = st.watermarks;
    if (nw > gw_handle::kNbWmHost) {
        wpos.resize(nw);
        wval.resize(nw);
        e = hipMemcpy(wpos.data(), wp, nw * 8, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(wval.data(), wv, nw * 8, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return h->fail(GW_E_DEVICE, "watermark list: %s", hipGetErrorString(e));
    } else {
        wpos.assign(h->h_nbwm, h->h_nbwm + nw);
        wval.assign(h->h_nbwm + gw_handle::kNbWmHost, h->h_nbwm + gw_handle::kNbWmHost + nw);
    }
    int64_t fired = 0, done = 0;
    for (int64_t i = 0; i <= nw; ++i) {
        const int64_t upto = i < nw ? wpos[i] : st.records;
        if (upto > done) {
            rc = ingest_device_impl(h, upto - done, k + done, t + done, L.val_type ? v + done : nullptr);
            if (rc) return rc;
            done = upto;
        }
        if (i < nw) {
            int64_t f = 0;
            rc = gw_advance_watermark(h, wval[i], &f);
            if (rc) return rc;
            fired += f;
        }
    }
    if (consumed) *consumed = st.consumed;
    if (rows_fired) *rows_fired = fired;
    return GW_OK;
}

int gw_ingest_serialized_device(gw_handle* h, const void* d_bytes, int64_t nbytes, const gw_record_layout* layout,
                                void* stream, int64_t* consumed, int64_t* rows_fired) {
    if (!h) return GW_E_INVALID;
    if (h->fe) return h->fail(GW_E_UNSUPPORTED, "network-buffer ingest of first-element rows is not supported");
    if (!h->kids.empty()) {  // each child decodes the channel (same bytes consumed by all)
        int64_t sum = 0;
        for (gw_handle* kid : h->kids) {
            int64_t f = 0;
            const int rc = gw_ingest_serialized_device(kid, d_bytes, nbytes, layout, stream, consumed, &f);
            if (rc) return kid_rc(h, kid, rc);
            sum += f;
        }
        if (rows_fired) *rows_fired = sum;
        return GW_OK;
    }
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    NbLayout L{};
    std::string why;
    int rc = nb_layout(layout, h->cfg.agg, L, why);
    if (rc) return h->fail(rc, "%s", why.c_str());
    if (nbytes < 0 || (nbytes > 0 && !d_bytes) || ((uintptr_t)d_bytes & 3))
        return h->fail(GW_E_INVALID, "bad byte buffer (device pointer, 4-byte aligned)");
    if (consumed) *consumed = 0;
    if (rows_fired) *rows_fired = 0;
    if (nbytes == 0) return GW_OK;
    hipSetDevice(h->cfg.device);
    hipStream_t ps = (hipStream_t)stream;
    if (ps != h->stream) {
        hipEventRecord(h->ev_in, ps);
        hipStreamWaitEvent(h->stream, h->ev_in, 0);
    }
    // the decode has read the bytes once this returns (it synchronises the handle's stream)
    return nb_ingest_on_stream(h, (const uint8_t*)d_bytes, nbytes, L, consumed, rows_fired);
}

int gw_ingest_serialized(gw_handle* h, const void* bytes, int64_t nbytes, const gw_record_layout* layout,
                         int64_t* consumed, int64_t* rows_fired) {
    if (!h) return GW_E_INVALID;
    if (h->fe) return h->fail(GW_E_UNSUPPORTED, "network-buffer ingest of first-element rows is not supported");
    if (!h->kids.empty()) {
        int64_t sum = 0;
        for (gw_handle* kid : h->kids) {
            int64_t f = 0;
            const int rc = gw_ingest_serialized(kid, bytes, nbytes, layout, consumed, &f);
            if (rc) return kid_rc(h, kid, rc);
            sum += f;
        }
        if (rows_fired) *rows_fired = sum;
        return GW_OK;
    }
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    NbLayout L{};
    std::string why;
    int rc = nb_layout(layout, h->cfg.agg, L, why);
    if (rc) return h->fail(rc, "%s", why.c_str());
    if (nbytes < 0 || (nbytes > 0 && !bytes)) return h->fail(GW_E_INVALID, "null byte buffer");
    if (consumed) *consumed = 0;
    if (rows_fired) *rows_fired = 0;
    if (nbytes == 0) return GW_OK;
    hipSetDevice(h->cfg.device);
    if (nbytes > h->nb_bytes_cap) {
        if (h->h_nbbytes) { hipHostFree(h->h_nbbytes); hipFree(h->d_nbbytes); }
        h->h_nbbytes = nullptr;
        h->d_nbbytes = nullptr;
        h->nb_bytes_cap = 0;
        const int64_t cap = std::max<int64_t>(nbytes, 1 << 20);
        hipError_t e = hipHostMalloc((void**)&h->h_nbbytes, (size_t)cap, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc((void**)&h->d_nbbytes, (size_t)cap);
        if (e != hipSuccess) return h->fail(GW_E_OOM, "network-buffer staging: %s", hipGetErrorString(e));
        h->nb_bytes_cap = cap;
    }
    // the previous call synchronised the stream, so the pinned staging is free
    memcpy(h->h_nbbytes, bytes, (size_t)nbytes);
    hipError_t e = hipMemcpyAsync(h->d_nbbytes, h->h_nbbytes, (size_t)nbytes, hipMemcpyHostToDevice, h->stream);
    if (e != hipSuccess) return h->fail(GW_E_DEVICE, "H2D: %s", hipGetErrorString(e));
    return nb_ingest_on_stream(h, h->d_nbbytes, nbytes, L, consumed, rows_fired);
}

int gw_advance_watermark(gw_handle* h, int64_t wm, int64_t* rows_fired) {
    if (!h) return GW_E_INVALID;
    if (h->fe) {  // both operators fire the same windows; join their rows now, while the log holds them
        int64_t f = 0;
        for (gw_handle* kid : h->kids) {
            const int rc = gw_advance_watermark(kid, wm, kid == h->kids[0] ? &f : nullptr);
            if (rc) return kid_rc(h, kid, rc);
        }
        if (wm > h->fe_wm) h->fe_wm = wm;
        if (f > 0) {  // both operators fired the same windows: join them, then release
            int rc = fe_gather(h);
            if (rc == GW_OK) rc = fe_release(h);
            if (rc) return rc;
        }
        h->stats.rows_fired += f;
        if (rows_fired) *rows_fired = f;
        return GW_OK;
    }
    if (!h->kids.empty()) {
        int64_t sum = 0;
        for (gw_handle* kid : h->kids) {
            int64_t f = 0;
            const int rc = gw_advance_watermark(kid, wm, &f);
            if (rc) return kid_rc(h, kid, rc);
            sum += f;
        }
        h->stats.rows_fired += sum;
        if (rows_fired) *rows_fired = sum;
        return GW_OK;
    }
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    hipSetDevice(h->cfg.device);
    if (h->session) {
        int64_t fired = 0;
        int rc = GW_OK;
        if (wm > h->wm) {
            rc = session_fire(h->sess, wm, &fired, h->err);
            if (rc == GW_OK) h->wm = wm;
            else if (rc == GW_E_DEVICE) h->failed = true;
        }
        h->stats.rows_fired += fired;
        if (rows_fired) *rows_fired = fired;
        return rc;
    }
    h->hp.mark();
    const int rc = h->advance_pane(wm, rows_fired);
    h->hp.lap(14);
    return rc;
}

int gw_flush(gw_handle* h) {
    if (!h) return GW_E_INVALID;
    if (!h->kids.empty()) {
        FOR_KIDS(gw_flush(kid));
        return GW_OK;
    }
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    if (h->session) return GW_OK;
    hipSetDevice(h->cfg.device);
    int rc = h->ov_finalize();
    if (rc == GW_OK) rc = h->ensure_fresh();
    return rc ? rc : h->flush_buffer();
}

// Window-class composite snapshots: the children's heap-layout blobs merged per key group
// (their (window, key, state) entries and timers are disjoint by window), under the
// composite's own assigner header; restore splits each key group's entries and timers by
// the class of their window.  Layout per key group (snapshot_heap): be32 n + n entries of
// (start, end, key, state), be32 0 (no merging window set), be32 t + t timers of 32 bytes.
typedef gw_handle::SnapHeader SnapHdr;
static int64_t comp_slide(const gw_handle* h) { return h->cfg.assigner == GW_TUMBLING ? h->cfg.size : h->cfg.slide; }
static int comp_snapshot(gw_handle* h, int32_t kg_lo, int32_t kg_hi, void* buf, int64_t cap, int64_t* len) {
    const int64_t nk = (int64_t)kg_hi - kg_lo + 1;
    if (kg_lo < 0 || nk <= 0) return h->fail(GW_E_INVALID, "bad key-group range");
    std::vector<std::vector<uint8_t>> blobs(h->kids.size());
    int64_t flags = -1;
    for (size_t j = 0; j < h->kids.size(); ++j) {
        int64_t l = 0;
        int rc = gw_snapshot(h->kids[j], kg_lo, kg_hi, nullptr, 0, &l);
        if (rc) return kid_rc(h, h->kids[j], rc);
        blobs[j].resize((size_t)l);
        if ((rc = gw_snapshot(h->kids[j], kg_lo, kg_hi, blobs[j].data(), l, &l))) return kid_rc(h, h->kids[j], rc);
        SnapHdr kh;
        memcpy(&kh, blobs[j].data(), sizeof kh);
        if (flags >= 0 && kh.flags != flags) return h->fail(GW_E_STATE, "window classes disagree on key hashes");
        flags = kh.flags;
    }
    // every class sees every batch, so all or none carry key hashes
    const int64_t eb = 24 + ((flags & kSnapKeyHashes) ? 4 : 0) + h->kids[0]->acc_bytes();
    std::vector<uint8_t> pay;
    std::vector<int64_t> offs(nk + 1, 0);
    const int64_t hb = (int64_t)sizeof(SnapHdr) + (nk + 1) * 8;
    for (int64_t g = 0; g < nk; ++g) {
        offs[g] = (int64_t)pay.size();
        // entries in snapshot_heap's order: by key, then window; timers by key, window, time
        std::vector<std::pair<std::pair<int64_t, int64_t>, const uint8_t*>> st;
        std::vector<std::pair<std::tuple<int64_t, int64_t, uint64_t>, const uint8_t*>> tm;
        for (auto& b : blobs) {
            int64_t o0;
            memcpy(&o0, b.data() + sizeof(SnapHdr) + g * 8, 8);
            const uint8_t* p = b.data() + hb + o0;
            const int32_t n = gw_handle::rd32(p);
            p += 4;
            for (int32_t i = 0; i < n; ++i, p += eb) st.push_back({{gw_handle::rd64(p + 16), gw_handle::rd64(p)}, p});
            p += 4;  // the empty merging window set
            const int32_t t = gw_handle::rd32(p);
            p += 4;
            for (int32_t i = 0; i < t; ++i, p += 32)
                tm.push_back({{gw_handle::rd64(p + 8), gw_handle::rd64(p + 16), (uint64_t)gw_handle::rd64(p)}, p});
        }
        std::sort(st.begin(), st.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        std::sort(tm.begin(), tm.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
        gw_handle::be32(pay, (int32_t)st.size());
        for (auto& e : st) pay.insert(pay.end(), e.second, e.second + eb);
        gw_handle::be32(pay, 0);
        gw_handle::be32(pay, (int32_t)tm.size());
        for (auto& e : tm) pay.insert(pay.end(), e.second, e.second + 32);
    }
    offs[nk] = (int64_t)pay.size();
    const int64_t need = hb + (int64_t)pay.size();
    *len = need;
    if (!buf) return GW_OK;
    if (cap < need) return h->fail(GW_E_OUTPUT_FULL, "snapshot needs %lld bytes", (long long)need);
    SnapHdr hd;
    memcpy(&hd, blobs[0].data(), sizeof hd);
    hd.assigner = h->cfg.assigner;
    hd.slide = comp_slide(h);
    hd.offset = h->cfg.offset;
    hd.entries = (int64_t)pay.size();
    char* out = (char*)buf;
    memcpy(out, &hd, sizeof hd);
    memcpy(out + sizeof hd, offs.data(), (size_t)(nk + 1) * 8);
    if (!pay.empty()) memcpy(out + hb, pay.data(), pay.size());
    return GW_OK;
}

static int restore_any(gw_handle* h, const void* buf, int64_t len, bool dry);

// Window classes: the blob is cut into one part per class; every part is checked (a dry
// restore) before any class restores, so a rejected blob leaves every class as it was.
static int comp_restore(gw_handle* h, const void* buf, int64_t len, bool dry) {
    if (!buf || len < (int64_t)sizeof(SnapHdr)) return h->fail(GW_E_INVALID, "snapshot blob too short");
    SnapHdr hd;
    memcpy(&hd, buf, sizeof hd);
    if (memcmp(hd.magic, "GWS1", 4) != 0 || hd.version != 4 || hd.agg != h->cfg.agg ||
        hd.assigner != h->cfg.assigner || hd.size != h->cfg.size || hd.slide != comp_slide(h) ||
        hd.offset != h->cfg.offset || hd.max_parallelism != h->cfg.max_parallelism)
        return h->fail(GW_E_INVALID, "snapshot of a different window / aggregate / max parallelism");
    const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
    const int64_t hb = (int64_t)sizeof hd + (nk + 1) * 8;
    if (nk <= 0 || hd.entries < 0 || len < hb || hd.entries > len - hb)
        return h->fail(GW_E_INVALID, "truncated snapshot blob");
    const int64_t J = (int64_t)h->kids.size();
    const int64_t eb = 24 + ((hd.flags & kSnapKeyHashes) ? 4 : 0) + h->kids[0]->acc_bytes();
    const uint8_t* p = (const uint8_t*)buf + hb;
    const uint8_t* end = p + hd.entries;
    auto cls = [&](int64_t s0) {  // window class of a window start
        const int64_t k = (int64_t)floor_div((i128)s0 - h->cfg.offset, (i128)comp_slide(h));
        return (size_t)(((k % J) + J) % J);
    };
    std::vector<std::vector<uint8_t>> pay(J);
    std::vector<std::vector<int64_t>> offs(J, std::vector<int64_t>(nk + 1, 0));
    for (int64_t g = 0; g < nk; ++g) {
        std::vector<std::vector<uint8_t>> st(J), tm(J);
        std::vector<int32_t> nst(J, 0), ntm(J, 0);
        if (end - p < 4) return h->fail(GW_E_INVALID, "truncated snapshot blob");
        const int32_t n = gw_handle::rd32(p);
        p += 4;
        if (n < 0 || (int64_t)n * eb + 8 > end - p) return h->fail(GW_E_INVALID, "truncated snapshot blob");
        for (int32_t i = 0; i < n; ++i, p += eb) {
            const size_t j = cls(gw_handle::rd64(p));
            st[j].insert(st[j].end(), p, p + eb);
            nst[j]++;
        }
        if (gw_handle::rd32(p) != 0) return h->fail(GW_E_INVALID, "merging window set in a sliding snapshot");
        p += 4;
        const int32_t t = gw_handle::rd32(p);
        p += 4;
        if (t < 0 || (int64_t)t * 32 > end - p) return h->fail(GW_E_INVALID, "truncated snapshot blob");
        for (int32_t i = 0; i < t; ++i, p += 32) {
            const size_t j = cls(gw_handle::rd64(p + 16));  // (timestamp, key, start, end)
            tm[j].insert(tm[j].end(), p, p + 32);
            ntm[j]++;
        }
        for (int64_t j = 0; j < J; ++j) {
            offs[j][g] = (int64_t)pay[j].size();
            gw_handle::be32(pay[j], nst[j]);
            pay[j].insert(pay[j].end(), st[j].begin(), st[j].end());
            gw_handle::be32(pay[j], 0);
            gw_handle::be32(pay[j], ntm[j]);
            pay[j].insert(pay[j].end(), tm[j].begin(), tm[j].end());
        }
    }
    if (p != end) return h->fail(GW_E_INVALID, "snapshot blob has trailing bytes");
    std::vector<std::vector<uint8_t>> blobs(J);
    for (int64_t j = 0; j < J; ++j) {
        offs[j][nk] = (int64_t)pay[j].size();
        SnapHdr kh = hd;
        kh.assigner = h->kids[j]->cfg.assigner;
        kh.slide = h->kids[j]->cfg.slide;
        kh.offset = h->kids[j]->cfg.offset;
        kh.entries = (int64_t)pay[j].size();
        std::vector<uint8_t>& blob = blobs[j];
        blob.resize(sizeof kh + (nk + 1) * 8 + pay[j].size());
        memcpy(blob.data(), &kh, sizeof kh);
        memcpy(blob.data() + sizeof kh, offs[j].data(), (size_t)(nk + 1) * 8);
        if (!pay[j].empty()) memcpy(blob.data() + sizeof kh + (nk + 1) * 8, pay[j].data(), pay[j].size());
        const int rc = restore_any(h->kids[j], blob.data(), (int64_t)blob.size(), true);
        if (rc) return kid_rc(h, h->kids[j], rc);
    }
    if (dry) return GW_OK;
    for (int64_t j = 0; j < J; ++j) {  // checked above: only a device error can fail here
        const int rc = restore_any(h->kids[j], blobs[j].data(), (int64_t)blobs[j].size(), false);
        if (rc) return kid_rc(h, h->kids[j], rc);
    }
    return GW_OK;
}

#define HIPCHECK_H(h, x)                                                                                  \
    do {                                                                                                  \
        hipError_t e_ = (x);                                                                              \
        if (e_ != hipSuccess) return (h)->fail(GW_E_DEVICE, "%s failed: %s", #x, hipGetErrorString(e_)); \
    } while (0)

// ---- first-element handles: one heap-layout blob for both operators -------------------
// The reference keeps one reduced Tuple per (key, window): the window's first element with
// the aggregated field replaced (HeapReducingState.java:90-97, SumAggregator /
// ComparableAggregator).  The blob holds exactly that per entry: (window, key, [hash],
// aggregate, payload of the first element) with flags |= kSnapFirstElement, and kids[0]'s
// timers.  A restore gives the restored first elements new arrival sequences: their payloads
// go to the log, kids[1] gets (window, key, new sequence) entries.
// minBy / maxBy handles hold the same entries: the element's payload comes from the log
// (fe_by_select over the entries' (key, window, MIN / MAX)) instead of kids[1]'s sequence.
static int fe_snapshot(gw_handle* h, int32_t kg_lo, int32_t kg_hi, void* buf, int64_t cap, int64_t* len) {
    gw_handle *A = h->kids[0], *B = h->fe_by ? h->kids[0] : h->kids[1];
    std::vector<uint8_t> ba, bb;
    for (auto pr : {std::make_pair(A, &ba), std::make_pair(B, &bb)}) {
        if (h->fe_by && pr.second == &bb) {
            bb = ba;
            break;
        }
        int64_t l = 0;
        int rc = gw_snapshot(pr.first, kg_lo, kg_hi, nullptr, 0, &l);
        if (rc) return kid_rc(h, pr.first, rc);
        pr.second->resize((size_t)l);
        if ((rc = gw_snapshot(pr.first, kg_lo, kg_hi, pr.second->data(), l, &l))) return kid_rc(h, pr.first, rc);
    }
    SnapHdr ha, hb;
    memcpy(&ha, ba.data(), sizeof ha);
    memcpy(&hb, bb.data(), sizeof hb);
    if (ha.version != 4 || hb.version != 4 || ha.flags != hb.flags)
        return h->fail(GW_E_STATE, "first-element snapshot: the operators' blobs differ");
    const int64_t nk = (int64_t)kg_hi - kg_lo + 1, hdr = (int64_t)sizeof(SnapHdr) + (nk + 1) * 8;
    const int kb = (ha.flags & kSnapKeyHashes) ? 4 : 0;
    const int64_t ea = 24 + kb + A->acc_bytes(), eb = 24 + kb + 8;  // B: MIN_I64 of the sequence
    // pass 1: the sequences of every entry's first element, in entry order
    std::vector<int64_t> seqs, by_key, by_start, by_res;
    struct Sec { const uint8_t *sa, *sb, *ta; int32_t n, t; };
    std::vector<Sec> secs((size_t)nk);
    for (int64_t g = 0; g < nk; ++g) {
        int64_t oa, ob;
        memcpy(&oa, ba.data() + sizeof(SnapHdr) + g * 8, 8);
        memcpy(&ob, bb.data() + sizeof(SnapHdr) + g * 8, 8);
        const uint8_t* pa = ba.data() + hdr + oa;
        const uint8_t* pb = bb.data() + hdr + ob;
        Sec sc{};
        sc.n = gw_handle::rd32(pa);
        if (gw_handle::rd32(pb) != sc.n) return h->fail(GW_E_STATE, "first-element snapshot: entries differ");
        sc.sa = pa + 4;
        sc.sb = pb + 4;
        for (int32_t i = 0; i < sc.n; ++i) {
            const uint8_t* xa = sc.sa + i * ea;
            const uint8_t* xb = sc.sb + i * eb;
            if (memcmp(xa, xb, 24 + kb) != 0) return h->fail(GW_E_STATE, "first-element snapshot: entries differ");
            if (h->fe_by) {  // (start, end, key, [hash], MIN / MAX)
                by_start.push_back(gw_handle::rd64(xa));
                by_key.push_back(gw_handle::rd64(xa + 16));
                by_res.push_back(gw_handle::rd64(xa + 24 + kb));
            } else {
                seqs.push_back(gw_handle::rd64(xb + 24 + kb));
            }
        }
        sc.ta = sc.sa + sc.n * ea + 4;  // past the (empty) merging window set
        sc.t = gw_handle::rd32(sc.ta);
        sc.ta += 4;
        secs[g] = sc;
    }
    std::vector<int64_t> pays(h->fe_by ? by_key.size() : seqs.size());
    if (h->fe_by && !by_key.empty()) {
        const size_t m = by_key.size();
        int64_t* d = nullptr;
        HIPCHECK_H(h, hipMalloc((void**)&d, m * 32));
        hipError_t e = hipMemcpyAsync(d, by_key.data(), m * 8, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(d + m, by_start.data(), m * 8, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(d + 2 * m, by_res.data(), m * 8, hipMemcpyHostToDevice, h->stream);
        int rc = e == hipSuccess ? by_select(h, (int64_t)m, d, d + m, d + 2 * m, nullptr, d + 3 * m)
                                 : h->fail(GW_E_DEVICE, "minBy / maxBy snapshot: %s", hipGetErrorString(e));
        if (rc == GW_OK && hipMemcpy(pays.data(), d + 3 * m, m * 8, hipMemcpyDeviceToHost) != hipSuccess)
            rc = h->fail(GW_E_DEVICE, "minBy / maxBy snapshot");
        hipFree(d);
        if (rc) return rc;
    }
    if (!seqs.empty()) {
        for (int64_t q : seqs)
            if (q < h->fe_log_base || q >= h->fe_seq) return h->fail(GW_E_STATE, "first-element snapshot: payload released");
        int64_t* d = nullptr;
        HIPCHECK_H(h, hipMalloc((void**)&d, seqs.size() * 16));
        hipError_t e = hipMemcpyAsync(d, seqs.data(), seqs.size() * 8, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = fe_log_gather(h->fe_log, h->fe_log_cap, d, (int64_t)seqs.size(), d + seqs.size(), h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(pays.data(), d + seqs.size(), seqs.size() * 8, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        hipFree(d);
        if (e != hipSuccess) return h->fail(GW_E_DEVICE, "first-element snapshot: %s", hipGetErrorString(e));
    }
    // pass 2: the blob
    std::vector<uint8_t> pay;
    std::vector<int64_t> offs(nk + 1, 0);
    size_t q = 0;
    for (int64_t g = 0; g < nk; ++g) {
        const Sec& sc = secs[g];
        offs[g] = (int64_t)pay.size();
        gw_handle::be32(pay, sc.n);
        for (int32_t i = 0; i < sc.n; ++i) {
            const uint8_t* xa = sc.sa + i * ea;
            pay.insert(pay.end(), xa, xa + ea);
            gw_handle::be64(pay, pays[q++]);
        }
        gw_handle::be32(pay, 0);
        gw_handle::be32(pay, sc.t);
        pay.insert(pay.end(), sc.ta, sc.ta + (size_t)sc.t * 32);
    }
    offs[nk] = (int64_t)pay.size();
    *len = hdr + (int64_t)pay.size();
    if (!buf) return GW_OK;
    if (cap < *len) return h->fail(GW_E_OUTPUT_FULL, "snapshot needs %lld bytes", (long long)*len);
    SnapHdr hd = ha;
    hd.agg = h->cfg.agg;
    hd.flags |= kSnapFirstElement;
    hd.entries = (int64_t)pay.size();
    char* out = (char*)buf;
    memcpy(out, &hd, sizeof hd);
    memcpy(out + sizeof hd, offs.data(), (size_t)(nk + 1) * 8);
    if (!pay.empty()) memcpy(out + hdr, pay.data(), pay.size());
    return GW_OK;
}

static int fe_restore(gw_handle* h, const void* buf, int64_t len, bool dry) {
    if (!buf || len < (int64_t)sizeof(SnapHdr)) return h->fail(GW_E_INVALID, "snapshot blob too short");
    SnapHdr hd;
    memcpy(&hd, buf, sizeof hd);
    if (memcmp(hd.magic, "GWS1", 4) != 0 || hd.version != 4 || !(hd.flags & kSnapFirstElement) || hd.agg != h->cfg.agg)
        return h->fail(GW_E_INVALID, "not a first-element snapshot of this aggregate");
    gw_handle *A = h->kids[0], *B = h->fe_by ? nullptr : h->kids[1];
    const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1, hdr = (int64_t)sizeof hd + (nk + 1) * 8;
    if (nk <= 0 || hd.entries < 0 || len < hdr || hd.entries > len - hdr)
        return h->fail(GW_E_INVALID, "truncated snapshot blob");
    std::vector<int64_t> by_cols[3];  // minBy / maxBy: the restored elements' key, window start, field
    const int kb = (hd.flags & kSnapKeyHashes) ? 4 : 0;
    const int64_t ea = 24 + kb + A->acc_bytes(), ef = ea + 8;
    const uint8_t* p = (const uint8_t*)buf + hdr;
    const uint8_t* end = p + hd.entries;
    std::vector<uint8_t> pa, pb;
    std::vector<int64_t> oa(nk + 1), ob(nk + 1), pays;
    int64_t max_end = INT64_MIN;
    const int64_t seq0 = h->fe_seq;
    for (int64_t g = 0; g < nk; ++g) {
        oa[g] = (int64_t)pa.size();
        ob[g] = (int64_t)pb.size();
        if (end - p < 4) return h->fail(GW_E_INVALID, "truncated snapshot blob");
        const int32_t n = gw_handle::rd32(p);
        p += 4;
        if (n < 0 || (int64_t)n * ef + 8 > end - p) return h->fail(GW_E_INVALID, "truncated snapshot blob");
        gw_handle::be32(pa, n);
        gw_handle::be32(pb, n);
        for (int32_t i = 0; i < n; ++i, p += ef) {
            pa.insert(pa.end(), p, p + ea);
            pb.insert(pb.end(), p, p + 24 + kb);
            gw_handle::be64(pb, seq0 + (int64_t)pays.size());  // the restored first element's new sequence
            pays.push_back(gw_handle::rd64(p + ea));
            max_end = std::max(max_end, gw_handle::rd64(p + 8));
            if (h->fe_by) {
                by_cols[0].push_back(gw_handle::rd64(p + 16));
                by_cols[1].push_back(gw_handle::rd64(p));
                by_cols[2].push_back(gw_handle::rd64(p + 24 + kb));
            }
        }
        if (gw_handle::rd32(p) != 0) return h->fail(GW_E_INVALID, "merging window set in a first-element snapshot");
        p += 4;
        const int32_t t = gw_handle::rd32(p);
        p += 4;
        if (t < 0 || (int64_t)t * 32 > end - p) return h->fail(GW_E_INVALID, "truncated snapshot blob");
        for (std::vector<uint8_t>* v : {&pa, &pb}) {
            gw_handle::be32(*v, 0);
            gw_handle::be32(*v, t);
            v->insert(v->end(), p, p + (size_t)t * 32);
        }
        p += (size_t)t * 32;
    }
    if (p != end) return h->fail(GW_E_INVALID, "snapshot blob has trailing bytes");
    oa[nk] = (int64_t)pa.size();
    ob[nk] = (int64_t)pb.size();
    // the two operators' blobs, each checked (a dry restore: header, windows, counts, key
    // hashes, restore before processing) before the log or any operator changes
    std::vector<uint8_t> blobs[2];
    for (int w = 0; w < (h->fe_by ? 1 : 2); ++w) {
        std::vector<uint8_t>& pl = w ? pb : pa;
        std::vector<int64_t>& of = w ? ob : oa;
        SnapHdr kh = hd;
        kh.flags &= ~kSnapFirstElement;
        kh.agg = w ? GW_MIN_I64 : h->cfg.agg;
        kh.entries = (int64_t)pl.size();
        std::vector<uint8_t>& blob = blobs[w];
        blob.resize(sizeof kh + (size_t)(nk + 1) * 8 + pl.size());
        memcpy(blob.data(), &kh, sizeof kh);
        memcpy(blob.data() + sizeof kh, of.data(), (size_t)(nk + 1) * 8);
        if (!pl.empty()) memcpy(blob.data() + sizeof kh + (nk + 1) * 8, pl.data(), pl.size());
        gw_handle* kid = w ? B : A;
        const int rc = restore_any(kid, blob.data(), (int64_t)blob.size(), true);
        if (rc) return kid_rc(h, kid, rc);
    }
    if (dry) return GW_OK;
    // the payloads enter the log as one batch released once every restored window is cleaned
    const int64_t m = (int64_t)pays.size();
    if (m) {
        int rc = fe_log_reserve(h, m);
        if (rc) return rc;
        int64_t* d = nullptr;
        HIPCHECK_H(h, hipMalloc((void**)&d, (size_t)m * 8 * h->fe_cols));
        hipError_t e = hipMemcpy(d, pays.data(), (size_t)m * 8, hipMemcpyHostToDevice);
        for (int c = 1; c < h->fe_cols && e == hipSuccess; ++c)
            e = hipMemcpy(d + c * m, by_cols[c - 1].data(), (size_t)m * 8, hipMemcpyHostToDevice);
        for (int c = 0; c < h->fe_cols && e == hipSuccess; ++c)
            e = fe_log_append(h->fe_log + c * h->fe_log_cap, h->fe_log_cap, h->fe_seq, d + c * m, m, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        hipFree(d);
        if (e != hipSuccess) return h->fail(GW_E_DEVICE, "first-element restore: %s", hipGetErrorString(e));
        h->fe_seq += m;
        if (h->fe_by) h->fe_restored_end = h->fe_seq;  // restored elements stand for their own window
        // released like a batch whose records reach the latest restored window: maxTs + size - 1 = its end - 1
        h->fe_batches.push_back({h->fe_seq, 0, max_end - h->cfg.size, true});
    }
    for (int w = 0; w < (h->fe_by ? 1 : 2); ++w) {  // checked above: only a device error can fail here
        gw_handle* kid = w ? B : A;
        const int rc = restore_any(kid, blobs[w].data(), (int64_t)blobs[w].size(), false);
        if (rc) return kid_rc(h, kid, rc);
    }
    return GW_OK;
}

int gw_snapshot(gw_handle* h, int32_t kg_lo, int32_t kg_hi, void* buf, int64_t cap, int64_t* len) {
    if (!h || !len) return GW_E_INVALID;
    if (h->fe) return fe_snapshot(h, kg_lo, kg_hi, buf, cap, len);
    if (!h->kids.empty()) return comp_snapshot(h, kg_lo, kg_hi, buf, cap, len);
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    hipSetDevice(h->cfg.device);
    if (h->session) return h->snapshot_sessions(kg_lo, kg_hi, buf, cap, len);
    return h->snapshot_heap(kg_lo, kg_hi, buf, cap, len);
}

static int restore_any(gw_handle* h, const void* buf, int64_t len, bool dry) {
    if (h->fe) return fe_restore(h, buf, len, dry);
    if (!h->kids.empty()) return comp_restore(h, buf, len, dry);
    if (h->failed) return h->fail(GW_E_STATE, "operator failed earlier: %s", h->err.c_str());
    hipSetDevice(h->cfg.device);
    if (h->session) return h->restore_sessions(buf, len, dry);
    return h->restore_heap(buf, len, dry);
}

int gw_restore(gw_handle* h, const void* buf, int64_t len) {
    if (!h) return GW_E_INVALID;
    return restore_any(h, buf, len, false);
}

// The blob layout is gw_handle::SnapHeader (96 bytes: kg_lo at 60, kg_hi at 64, reserved at
// 68, entries at 88), kg_offsets[kg_hi - kg_lo + 2], then the entries; an entry is 32 bytes in
// version 1 and `reserved` int64 words in every later version.
int gw_snapshot_slice(const void* blob, int64_t len, int32_t kg, void* out, int64_t cap, int64_t* out_len) {
    typedef gw_handle::SnapHeader H;
    static_assert(sizeof(H) == 96, "snapshot header layout");
    if (!blob || !out_len || len < (int64_t)sizeof(H)) { g_create_error = "snapshot blob too short"; return GW_E_INVALID; }
    H hd;
    memcpy(&hd, blob, sizeof hd);
    if (memcmp(hd.magic, "GWS1", 4) != 0 || hd.version < 1 || hd.version > kSnapMaxVersion) {
        g_create_error = "not a gpuwin snapshot";
        return GW_E_INVALID;
    }
    const int64_t ew = hd.version == 1 ? 32 : hd.version >= 4 ? 1 : (int64_t)hd.reserved * 8;  // v4: bytes
    const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
    if (ew <= 0 || nk <= 0 || hd.entries < 0 || len < (int64_t)sizeof hd + (nk + 1) * 8 ||
        hd.entries > (len - (int64_t)sizeof hd - (nk + 1) * 8) / ew) {
        g_create_error = "truncated snapshot blob";
        return GW_E_INVALID;
    }
    if (kg < hd.kg_lo || kg > hd.kg_hi) {
        g_create_error = "key group outside the blob's key-group range";
        return GW_E_INVALID;
    }
    const char* b = (const char*)blob;
    int64_t o0, o1;
    memcpy(&o0, b + sizeof hd + (kg - hd.kg_lo) * 8, 8);
    memcpy(&o1, b + sizeof hd + (kg - hd.kg_lo + 1) * 8, 8);
    if (o0 < 0 || o1 < o0 || o1 > hd.entries) { g_create_error = "corrupt snapshot offsets"; return GW_E_INVALID; }
    const int64_t n = o1 - o0;
    const int64_t need = (int64_t)sizeof hd + 16 + n * ew;
    *out_len = need;
    if (!out) return GW_OK;
    if (cap < need) { g_create_error = "slice buffer too small"; return GW_E_OUTPUT_FULL; }
    H oh = hd;
    oh.kg_lo = oh.kg_hi = kg;
    oh.entries = n;
    char* o = (char*)out;
    memcpy(o, &oh, sizeof oh);
    const int64_t offs[2] = {0, n};
    memcpy(o + sizeof oh, offs, 16);
    if (n) memcpy(o + sizeof oh + 16, b + sizeof hd + (nk + 1) * 8 + o0 * ew, (size_t)(n * ew));
    return GW_OK;
}

extern "C++" {
// Calls f(p, big_endian) for the key field of every entry, merging-set key and timer of a
// version 2-4 blob; false for a corrupt blob.
template <class F>
static bool blob_keys(const uint8_t* b, int64_t len, F&& f) {
    typedef gw_handle::SnapHeader H;
    H hd;
    if (!b || len < (int64_t)sizeof hd) return false;
    memcpy(&hd, b, sizeof hd);
    if (memcmp(hd.magic, "GWS1", 4) != 0 || hd.version < 2 || hd.version > kSnapMaxVersion) return false;
    const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1;
    const int64_t pay0 = (int64_t)sizeof hd + (nk + 1) * 8;
    if (nk <= 0 || hd.entries < 0 || len < pay0) return false;
    const uint8_t* p = b + pay0;
    if (hd.version < 4) {  // fixed entries of `reserved` int64 words, key first
        const int64_t ew = (int64_t)hd.reserved * 8;
        if (ew <= 0 || hd.entries > (len - pay0) / ew) return false;
        for (int64_t i = 0; i < hd.entries; ++i) f(p + i * ew, false);
        return true;
    }
    if (hd.entries > len - pay0) return false;
    const uint8_t* end = p + hd.entries;
    const int64_t ab = hd.agg == GW_SUM_I32 ? 4 : (hd.agg == GW_AVG_I64 || hd.agg == GW_AVG_F64) ? 16 : 8;
    if (hd.assigner == GW_COUNT_TUMBLING) {  // (GlobalWindow byte, key, [hash,] state) and (byte, key, [hash,] count)
        const int64_t hb = (hd.flags & kSnapKeyHashes) ? 4 : 0;
        for (int64_t g = 0; g < nk; ++g) {
            for (int sec = 0; sec < 2; ++sec) {
                const int64_t eb = 9 + hb + (sec ? 8 : ab);
                if (end - p < 4) return false;
                const int32_t n = gw_handle::rd32(p);
                p += 4;
                if (n < 0 || (int64_t)n * eb > end - p) return false;
                for (int32_t i = 0; i < n; ++i, p += eb) f(p + 1, true);
            }
            if (end - p < 4 || gw_handle::rd32(p) != 0) return false;
            p += 4;
        }
        return p == end;
    }
    const int64_t eb = 24 + ((hd.flags & kSnapKeyHashes) ? 4 : 0) + ((hd.flags & kSnapFirstElement) ? 8 : 0) + ab;
    for (int64_t g = 0; g < nk; ++g) {
        if (end - p < 4) return false;
        const int32_t n = gw_handle::rd32(p);
        p += 4;
        if (n < 0 || (int64_t)n * eb + 4 > end - p) return false;
        for (int32_t i = 0; i < n; ++i, p += eb) f(p + 16, true);
        const int32_t m = gw_handle::rd32(p);
        p += 4;
        if (m < 0) return false;
        const int64_t mh = 12 + ((hd.flags & kSnapKeyHashes) ? 4 : 0);
        for (int32_t i = 0; i < m; ++i) {  // merging window sets: (key, [be32 hash,] be32 c, c x 32 B)
            if (end - p < mh) return false;
            const int32_t c = gw_handle::rd32(p + mh - 4);
            if (c < 0 || (int64_t)c * 32 > end - p - mh) return false;
            f(p, true);
            p += mh + (int64_t)c * 32;
        }
        if (end - p < 4) return false;
        const int32_t t = gw_handle::rd32(p);
        p += 4;
        if (t < 0 || (int64_t)t * 32 > end - p) return false;
        for (int32_t i = 0; i < t; ++i, p += 32) f(p + 8, true);
    }
    return p == end;
}

static int64_t key_at(const uint8_t* p, bool be) {
    if (be) return gw_handle::rd64(p);
    int64_t k;
    memcpy(&k, p, 8);
    return k;
}

}  // extern "C++"

extern "C++" {
// Calls f(payload field, window end) for every entry of a first-element blob; false for a
// corrupt blob or one without payloads.
template <class F>
static bool blob_payloads(const uint8_t* b, int64_t len, F&& f) {
    typedef gw_handle::SnapHeader H;
    H hd;
    if (!b || len < (int64_t)sizeof hd) return false;
    memcpy(&hd, b, sizeof hd);
    if (memcmp(hd.magic, "GWS1", 4) != 0 || hd.version != 4 || !(hd.flags & kSnapFirstElement)) return false;
    const int64_t acc = hd.agg == GW_SUM_I32 ? 4 : (hd.agg == GW_AVG_I64 || hd.agg == GW_AVG_F64) ? 16 : 8;
    const int64_t at = 24 + ((hd.flags & kSnapKeyHashes) ? 4 : 0) + acc, eb = at + 8;
    const int64_t nk = (int64_t)hd.kg_hi - hd.kg_lo + 1, pay0 = (int64_t)sizeof hd + (nk + 1) * 8;
    if (nk <= 0 || hd.entries < 0 || len < pay0 || hd.entries > len - pay0) return false;
    const uint8_t* p = b + pay0;
    const uint8_t* end = p + hd.entries;
    for (int64_t g = 0; g < nk; ++g) {
        if (end - p < 4) return false;
        const int32_t n = gw_handle::rd32(p);
        p += 4;
        if (n < 0 || (int64_t)n * eb + 8 > end - p) return false;
        for (int32_t i = 0; i < n; ++i, p += eb) f(p + at, gw_handle::rd64(p + 8));
        p += 4;  // (empty) merging window set
        const int32_t t = gw_handle::rd32(p);
        p += 4;
        if (t < 0 || (int64_t)t * 32 > end - p) return false;
        p += (int64_t)t * 32;
    }
    return p == end;
}

}  // extern "C++"

int gw_snapshot_payloads(const void* blob, int64_t len, int64_t* payloads, int64_t cap, int64_t* n,
                         int64_t* max_window_end) {
    if (!n) return GW_E_INVALID;
    std::vector<int64_t> ps;
    int64_t mx = INT64_MIN;
    if (!blob_payloads((const uint8_t*)blob, len, [&](const uint8_t* p, int64_t e) {
            ps.push_back(gw_handle::rd64(p));
            mx = std::max(mx, e);
        })) {
        g_create_error = "not a first-element snapshot blob";
        return GW_E_INVALID;
    }
    std::sort(ps.begin(), ps.end());
    ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
    *n = (int64_t)ps.size();
    if (max_window_end) *max_window_end = mx;
    if (!payloads) return GW_OK;
    if (cap < *n) { g_create_error = "payload buffer too small"; return GW_E_OUTPUT_FULL; }
    if (!ps.empty()) memcpy(payloads, ps.data(), ps.size() * 8);
    return GW_OK;
}

int gw_snapshot_remap_payloads(void* blob, int64_t len, const int64_t* from, const int64_t* to, int64_t n) {
    if (n < 0 || (n > 0 && (!from || !to))) { g_create_error = "null payload map"; return GW_E_INVALID; }
    for (int64_t i = 1; i < n; ++i)
        if (from[i] <= from[i - 1]) { g_create_error = "remap payloads: from[] not ascending"; return GW_E_INVALID; }
    const bool ok = blob_payloads((const uint8_t*)blob, len, [&](const uint8_t* cp, int64_t) {
        uint8_t* p = const_cast<uint8_t*>(cp);
        const int64_t v = gw_handle::rd64(p);
        const int64_t* it = std::lower_bound(from, from + n, v);
        if (it == from + n || *it != v) return;
        const int64_t w = to[it - from];
        for (int i = 0; i < 8; ++i) p[i] = (uint8_t)((uint64_t)w >> (56 - 8 * i));
    });
    if (!ok) { g_create_error = "not a first-element snapshot blob"; return GW_E_INVALID; }
    return GW_OK;
}

int gw_snapshot_keys(const void* blob, int64_t len, int64_t* keys, int64_t cap, int64_t* n) {
    if (!n) return GW_E_INVALID;
    std::vector<int64_t> ks;
    if (!blob_keys((const uint8_t*)blob, len, [&](const uint8_t* p, bool be) { ks.push_back(key_at(p, be)); })) {
        g_create_error = "corrupt snapshot blob";
        return GW_E_INVALID;
    }
    std::sort(ks.begin(), ks.end());
    ks.erase(std::unique(ks.begin(), ks.end()), ks.end());
    *n = (int64_t)ks.size();
    if (!keys) return GW_OK;
    if (cap < *n) { g_create_error = "key buffer too small"; return GW_E_OUTPUT_FULL; }
    if (!ks.empty()) memcpy(keys, ks.data(), ks.size() * 8);
    return GW_OK;
}

int gw_snapshot_remap_keys(void* blob, int64_t len, const int64_t* from, const int64_t* to, int64_t n) {
    if (n < 0 || (n > 0 && (!from || !to))) { g_create_error = "null key map"; return GW_E_INVALID; }
    for (int64_t i = 1; i < n; ++i)
        if (from[i] <= from[i - 1]) { g_create_error = "remap keys: from[] not ascending"; return GW_E_INVALID; }
    const bool ok = blob_keys((const uint8_t*)blob, len, [&](const uint8_t* cp, bool be) {
        uint8_t* p = const_cast<uint8_t*>(cp);
        const int64_t k = key_at(p, be);
        const int64_t* it = std::lower_bound(from, from + n, k);
        if (it == from + n || *it != k) return;
        const int64_t v = to[it - from];
        if (be) {
            for (int i = 0; i < 8; ++i) p[i] = (uint8_t)((uint64_t)v >> (56 - 8 * i));
        } else {
            memcpy(p, &v, 8);
        }
    });
    if (!ok) { g_create_error = "corrupt snapshot blob"; return GW_E_INVALID; }
    return GW_OK;
}

int gw_end_input(gw_handle* h, int64_t* rows_fired) { return gw_advance_watermark(h, INT64_MAX, rows_fired); }

static void rows_view(gw_handle* h, int64_t** k, int64_t** s, int64_t** e, int64_t** r, int64_t* total) {
    if (h->session) {
        session_rows(h->sess, k, s, e, r, total);
    } else {
        *k = h->o_key; *s = h->o_start; *e = h->o_end; *r = h->o_res;
        *total = (int64_t)h->h_st->rows;
    }
}

int gw_pending_rows(gw_handle* h, int64_t* n) {
    if (!h || !n) return GW_E_INVALID;
    if (h->fe) {  // rows are joined at every watermark
        *n = h->c_rows - h->c_head;
        return GW_OK;
    }
    if (!h->kids.empty()) {
        int64_t sum = h->c_rows - h->c_head;
        for (gw_handle* kid : h->kids) {
            int64_t p = 0;
            const int rc = gw_pending_rows(kid, &p);
            if (rc) return kid_rc(h, kid, rc);
            sum += p;
        }
        *n = sum;
        return GW_OK;
    }
    int rc = h->session ? session_refresh(h->sess, h->err) : h->refresh();
    if (rc) return rc;
    int64_t *k, *s, *e, *r, total;
    rows_view(h, &k, &s, &e, &r, &total);
    *n = total - h->rows_head;
    return GW_OK;
}

int gw_drain(gw_handle* h, int64_t* key, int64_t* start, int64_t* end, void* result, int64_t cap,
             int64_t* n) {
    if (!h || !n) return GW_E_INVALID;
    if (h->fe) return gw_drain_payload(h, key, start, end, result, nullptr, cap, n);
    if (!h->kids.empty()) {  // the gathered rows first, then each child's
        int64_t got = 0;
        auto at = [&](int64_t* p) { return p ? p + got : nullptr; };
        const int64_t c = std::min(cap, h->c_rows - h->c_head);
        if (c > 0) {
            hipError_t e = hipSuccess;
            const int64_t o = h->c_head;
            if (key) e = hipMemcpyAsync(key, h->c_key + o, c * 8, hipMemcpyDeviceToHost, h->stream);
            if (start && e == hipSuccess) e = hipMemcpyAsync(start, h->c_start + o, c * 8, hipMemcpyDeviceToHost, h->stream);
            if (end && e == hipSuccess) e = hipMemcpyAsync(end, h->c_end + o, c * 8, hipMemcpyDeviceToHost, h->stream);
            if (result && e == hipSuccess)
                e = hipMemcpyAsync(result, h->c_res + o, c * 8, hipMemcpyDeviceToHost, h->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
            if (e != hipSuccess) return h->fail(GW_E_DEVICE, "D2H rows: %s", hipGetErrorString(e));
            h->c_head += c;
            got += c;
            if (h->c_head == h->c_rows) h->c_head = h->c_rows = 0;
        }
        for (gw_handle* kid : h->kids) {
            if (got == cap) break;
            int64_t g = 0;
            const int rc = gw_drain(kid, at(key), at(start), at(end), result ? (void*)((int64_t*)result + got) : nullptr,
                                    cap - got, &g);
            if (rc && rc != GW_E_OUTPUT_FULL) return kid_rc(h, kid, rc);
            got += g;
        }
        *n = got;
        int64_t left = 0;
        const int rc = gw_pending_rows(h, &left);
        if (rc) return rc;
        return left ? GW_E_OUTPUT_FULL : GW_OK;
    }
    int64_t pending;
    int rc = gw_pending_rows(h, &pending);
    if (rc) return rc;
    int64_t *k, *s, *e, *r, total;
    rows_view(h, &k, &s, &e, &r, &total);
    const int64_t c = std::min(cap, pending);
    const int64_t o = h->rows_head;
    if (c > 0) {
        int64_t* dst[4] = {key, start, end, (int64_t*)result};
        const int64_t* src[4] = {k + o, s + o, e + o, r + o};
        if ((rc = h->drain_to_host(dst, src, c))) return rc;
    }
    *n = c;
    h->rows_head += c;
    if (h->rows_head == total) {
        rc = gw_clear_rows(h);
        if (rc) return rc;
    }
    return c < pending ? GW_E_OUTPUT_FULL : GW_OK;
}

int gw_rows_device(gw_handle* h, const int64_t** d_key, const int64_t** d_start, const int64_t** d_end,
                   const void** d_result, int64_t* n) {
    if (!h) return GW_E_INVALID;
    if (h->fe) {
        const int64_t o = h->c_head;
        if (d_key) *d_key = h->c_key ? h->c_key + o : nullptr;
        if (d_start) *d_start = h->c_start ? h->c_start + o : nullptr;
        if (d_end) *d_end = h->c_end ? h->c_end + o : nullptr;
        if (d_result) *d_result = h->c_res ? h->c_res + o : nullptr;
        if (n) *n = h->c_rows - h->c_head;
        return GW_OK;
    }
    if (!h->kids.empty()) {  // gather the children's pending rows behind the waiting ones
        int64_t add = 0;
        for (gw_handle* kid : h->kids) {
            int64_t p = 0;
            const int rc = gw_pending_rows(kid, &p);
            if (rc) return kid_rc(h, kid, rc);
            add += p;
        }
        if (h->c_rows + add > h->c_cap) {
            const int64_t cap = std::max<int64_t>(h->c_rows + add, 2 * h->c_cap);
            int64_t* nb[4] = {nullptr, nullptr, nullptr, nullptr};
            for (int q = 0; q < 4; ++q) {
                hipError_t e = hipMalloc((void**)&nb[q], (size_t)cap * 8);
                if (e != hipSuccess) {
                    for (int r = 0; r < q; ++r) hipFree(nb[r]);
                    return h->fail(GW_E_OOM, "composite row buffer: %s", hipGetErrorString(e));
                }
            }
            int64_t* old[4] = {h->c_key, h->c_start, h->c_end, h->c_res};
            const int64_t live = h->c_rows - h->c_head;
            for (int q = 0; q < 4; ++q) {
                if (old[q] && live) hipMemcpyAsync(nb[q], old[q] + h->c_head, live * 8, hipMemcpyDeviceToDevice, h->stream);
                if (old[q]) { hipStreamSynchronize(h->stream); hipFree(old[q]); }
            }
            h->c_key = nb[0]; h->c_start = nb[1]; h->c_end = nb[2]; h->c_res = nb[3];
            h->c_cap = cap;
            h->c_rows = live;
            h->c_head = 0;
        }
        for (gw_handle* kid : h->kids) {
            const int64_t* k[4];
            int64_t p = 0;
            int rc = gw_rows_device(kid, &k[0], &k[1], &k[2], (const void**)&k[3], &p);
            if (rc) return kid_rc(h, kid, rc);
            int64_t* dst[4] = {h->c_key, h->c_start, h->c_end, h->c_res};
            for (int q = 0; q < 4 && p > 0; ++q) {
                hipError_t e = hipMemcpyAsync(dst[q] + h->c_rows, k[q], p * 8, hipMemcpyDeviceToDevice, h->stream);
                if (e != hipSuccess) return h->fail(GW_E_DEVICE, "gather rows: %s", hipGetErrorString(e));
            }
            h->c_rows += p;
            if ((rc = gw_clear_rows(kid))) return kid_rc(h, kid, rc);
        }
        const int64_t o = h->c_head;
        if (d_key) *d_key = h->c_key ? h->c_key + o : nullptr;
        if (d_start) *d_start = h->c_start ? h->c_start + o : nullptr;
        if (d_end) *d_end = h->c_end ? h->c_end + o : nullptr;
        if (d_result) *d_result = h->c_res ? h->c_res + o : nullptr;
        if (n) *n = h->c_rows - h->c_head;
        return GW_OK;
    }
    int64_t pending;
    int rc = gw_pending_rows(h, &pending);
    if (rc) return rc;
    int64_t *k, *s, *e, *r, total;
    rows_view(h, &k, &s, &e, &r, &total);
    const int64_t o = h->rows_head;
    if (d_key) *d_key = k ? k + o : nullptr;
    if (d_start) *d_start = s ? s + o : nullptr;
    if (d_end) *d_end = e ? e + o : nullptr;
    if (d_result) *d_result = r ? r + o : nullptr;
    if (n) *n = pending;
    return GW_OK;
}

int gw_clear_rows(gw_handle* h) {
    if (!h) return GW_E_INVALID;
    if (!h->kids.empty()) {
        h->c_rows = h->c_head = 0;
        FOR_KIDS(gw_clear_rows(kid));
        return GW_OK;
    }
    h->rows_head = 0;
    if (h->session) return session_clear_rows(h->sess, h->err);
    if (h->h_st->rows == 0) return GW_OK;  // rows only grow in a fire, which refreshes h_st
    h->h_st->rows = 0;  // the device cursor: by the next launch that emits rows (rows_reset_now)
    h->rows_reset_pending = true;
    return GW_OK;
}

int gw_pending_late(gw_handle* h, int64_t* n) {
    if (!h || !n) return GW_E_INVALID;
    *n = 0;
    if (h->fe) return gw_pending_late(h->kids[0], n);
    if (!h->kids.empty()) {
        for (gw_handle* kid : h->kids) {
            int64_t p = 0;
            const int rc = gw_pending_late(kid, &p);
            if (rc) return kid_rc(h, kid, rc);
            *n += p;
        }
        return GW_OK;
    }
    if (!(h->cfg.flags & GW_FLAG_LATE_SIDE_OUTPUT)) return GW_OK;
    if (h->session) return session_pending_late(h->sess, n, h->err);
    int rc = h->refresh();
    if (rc) return rc;
    *n = (int64_t)h->h_st->n_late_out - h->lo_head;
    return GW_OK;
}

int gw_drain_late(gw_handle* h, int64_t* key, int64_t* ts, void* value, int64_t cap, int64_t* n) {
    if (!h || !n) return GW_E_INVALID;
    *n = 0;
    if (h->fe) return gw_drain_late(h->kids[0], key, ts, value, cap, n);
    if (!h->kids.empty()) {  // each late record is reported by one child (its last window's class)
        int64_t got = 0;
        for (gw_handle* kid : h->kids) {
            if (got == cap) break;
            int64_t g = 0;
            const int rc = gw_drain_late(kid, key ? key + got : nullptr, ts ? ts + got : nullptr,
                                         value ? (void*)((int64_t*)value + got) : nullptr, cap - got, &g);
            if (rc && rc != GW_E_OUTPUT_FULL) return kid_rc(h, kid, rc);
            got += g;
        }
        *n = got;
        int64_t left = 0;
        const int rc = gw_pending_late(h, &left);
        if (rc) return rc;
        return left ? GW_E_OUTPUT_FULL : GW_OK;
    }
    if (!(h->cfg.flags & GW_FLAG_LATE_SIDE_OUTPUT)) return GW_OK;
    hipSetDevice(h->cfg.device);
    if (h->session) return session_drain_late(h->sess, key, ts, (int64_t*)value, cap, n, h->err);
    int64_t pending;
    int rc = gw_pending_late(h, &pending);
    if (rc) return rc;
    const int64_t c = std::min(cap, pending), o = h->lo_head;
    int64_t* dst[3] = {key, ts, (int64_t*)value};
    for (int q = 0; q < 3 && c > 0; ++q) {
        if (!dst[q]) continue;
        hipError_t e = hipMemcpyAsync(dst[q], h->lo_buf[q] + o, c * 8, hipMemcpyDeviceToHost, h->stream);
        if (e != hipSuccess) return h->fail(GW_E_DEVICE, "D2H late records: %s", hipGetErrorString(e));
    }
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return h->fail(GW_E_DEVICE, "D2H late records: %s", hipGetErrorString(e));
    *n = c;
    h->lo_head += c;
    if (c == pending) {  // emptied: restart the buffer
        h->lo_head = 0;
        h->lo_bound = 0;
        if (h->h_st->n_late_out && (rc = h->set_field(offsetof(DevStatus, n_late_out), 0))) return rc;
    }
    return c < pending ? GW_E_OUTPUT_FULL : GW_OK;
}

int64_t gw_late_dropped(const gw_handle* h) {
    if (!h) return 0;
    if (h->fe) return gw_late_dropped(h->kids[0]);
    if (!h->kids.empty()) {
        int64_t sum = 0;
        for (const gw_handle* kid : h->kids) sum += gw_late_dropped(kid);
        return sum;
    }
    if (h->session) return session_late(h->sess);
    return (int64_t)h->h_st->late;
}

int gw_get_stats(const gw_handle* h, gw_stats* out) {
    if (!h || !out) return GW_E_INVALID;
    if (h->fe) {
        gw_get_stats(h->kids[0], out);
        if (!h->fe_by) {
            gw_stats b{};
            gw_get_stats(h->kids[1], &b);
            out->table_bytes += b.table_bytes;
        }
        out->rows_fired = h->stats.rows_fired;
        return GW_OK;
    }
    if (!h->kids.empty()) {  // records: as one operator sees them; state: summed over the classes
        gw_stats t{};
        for (size_t j = 0; j < h->kids.size(); ++j) {
            gw_stats k{};
            gw_get_stats(h->kids[j], &k);
            if (j == 0) { t.events_in = k.events_in; t.batches = k.batches; }
            t.late_dropped += k.late_dropped;
            t.rows_fired += k.rows_fired;
            t.live_keys = std::max(t.live_keys, k.live_keys);
            t.table_capacity += k.table_capacity;
            t.table_bytes += k.table_bytes;
            t.deferred += k.deferred;
            t.fires += k.fires;
            t.rehashes += k.rehashes;
            t.preagg_batches += k.preagg_batches;
            t.applies += k.applies;
            t.region_format = k.region_format;
        }
        *out = t;
        return GW_OK;
    }
    *out = h->stats;
    if (h->session) {
        session_stats(h->sess, out);
    } else {
        out->late_dropped = (int64_t)h->h_st->late;
        out->live_keys = (int64_t)h->h_st->used_slots;
        out->deferred = (int64_t)h->h_st->n_deferred;
        out->table_capacity = h->tv.cap;
        out->table_bytes = (int64_t)h->table_bytes;
    }
    return GW_OK;
}

int gw_synchronize(gw_handle* h) {
    if (!h) return GW_E_INVALID;
    if (!h->kids.empty()) {
        FOR_KIDS(gw_synchronize(kid));
        return GW_OK;
    }
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return h->fail(GW_E_DEVICE, "sync: %s", hipGetErrorString(e));
    return GW_OK;
}

void* gw_stream(gw_handle* h) { return h ? (void*)h->stream : nullptr; }

int gw_enable_kernel_timing(gw_handle* h, int enable) {
    if (!h) return GW_E_INVALID;
    for (gw_handle* kid : h->kids) gw_enable_kernel_timing(kid, enable);
    h->timing = enable != 0;
    h->timing_every = enable > 1 ? enable : 1;
    h->timing_ctr = 0;
    if (h->sess) session_enable_timing(h->sess, h->timing);
    return GW_OK;
}

int gw_kernel_time_ms(gw_handle* h, int which, double* ms, int64_t* launches) {
    if (!h) return GW_E_INVALID;
    if (!h->kids.empty()) {  // per launch of child 0: the classes' device time together
        double total = 0;
        int64_t l0 = 0;
        for (size_t j = 0; j < h->kids.size(); ++j) {
            double m = 0;
            int64_t l = 0;
            gw_kernel_time_ms(h->kids[j], which, &m, &l);
            total += m * (double)l;
            if (j == 0) l0 = l;
        }
        if (ms) *ms = l0 ? total / (double)l0 : 0.0;
        if (launches) *launches = l0;
        return GW_OK;
    }
    hipStreamSynchronize(h->stream);
    if (h->sess) return session_kernel_time(h->sess, which, ms, launches);
    if (which == 3) {
        if (ms) *ms = 0.0;
        if (launches) *launches = h->fast_fires;
        return GW_OK;
    }
    KernelTimer& t = which == 0 ? h->t_ingest : which == 1 ? h->t_fire : h->t_apply;
    t.resolve();
    if (ms) *ms = t.launches ? t.total_ms / (double)t.launches : 0.0;
    if (launches) *launches = t.launches;
    t.total_ms = 0;
    t.launches = 0;
    return GW_OK;
}

// ---------------------------------------------------------------- window stagger
int gw_window_stagger_offset(int32_t stagger, int64_t processing_time, double random01, int64_t size,
                             int64_t global_offset, int64_t* offset_out) {
    if (!offset_out || size <= 0 || global_offset <= -size || global_offset >= size) return GW_E_INVALID;
    int64_t st = 0;
    switch (stagger) {
    case GW_STAGGER_ALIGNED: break;
    case GW_STAGGER_RANDOM:  // (long) (ThreadLocalRandom.current().nextDouble() * size)
        if (!(random01 >= 0.0 && random01 < 1.0)) return GW_E_INVALID;
        st = (int64_t)(random01 * (double)size);
        break;
    case GW_STAGGER_NATURAL: {  // currentProcessingTime - getWindowStartWithOffset(currentProcessingTime, 0, size)
        const int64_t rem = processing_time % size;
        const int64_t start = processing_time - (rem < 0 ? rem + size : rem);
        st = std::max<int64_t>(0, processing_time - start);
        break;
    }
    default: return GW_E_INVALID;
    }
    *offset_out = (global_offset + st) % size;  // both terms within (-size, size): no overflow
    return GW_OK;
}

// ---------------------------------------------------------------- key groups
int32_t gw_java_long_hash(int64_t key) { return java_long_hash(key); }
int32_t gw_murmur_hash(int32_t code) { return murmur_hash(code); }
int32_t gw_key_group_for_hash(int32_t h, int32_t max_p) { return key_group_for_hash(h, max_p); }
int32_t gw_operator_for_key_group(int32_t max_p, int32_t p, int32_t kg) { return operator_for_key_group(max_p, p, kg); }
int32_t gw_default_max_parallelism(int32_t p) {
    uint32_t u = (uint32_t)(p + p / 2) - 1u;
    u |= u >> 1; u |= u >> 2; u |= u >> 4; u |= u >> 8; u |= u >> 16;
    int32_t v = (int32_t)(u + 1u);
    return std::min(std::max(v, 128), 32768);
}

int gw_key_groups_device(int64_t n, const int64_t* d_key, const int32_t* d_key_hash, int32_t max_p, int32_t p,
                         int32_t* d_kg, int32_t* d_owner, void* stream) {
    if (n < 0 || max_p <= 0 || p <= 0 || p > max_p) return GW_E_INVALID;
    if (n == 0) return GW_OK;
    hipError_t e = launch_key_groups(n, d_key, d_key_hash, max_p, p, d_kg, d_owner, (hipStream_t)stream);
    if (e != hipSuccess) { g_create_error = hipGetErrorString(e); return GW_E_DEVICE; }
    return GW_OK;
}

int64_t gw_partition_scratch_bytes(int64_t n, int32_t p) { return partition_scratch_bytes(n, p); }

int gw_pack_records(int64_t n, const int64_t* key, const int64_t* ts, const int64_t* value, const gw_pack_geom* g,
                    uint64_t* words, uint8_t* fits) {
    if (n < 0 || !g || !g->enabled || g->pane <= 0 || (n > 0 && (!key || !ts || !words || !fits))) return GW_E_INVALID;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t w = 0;
        fits[i] = pack_word(*g, key[i], ts[i], value != nullptr, value ? value[i] : 0, w) ? 1 : 0;
        words[i] = fits[i] ? w : 0;
    }
    return GW_OK;
}

int gw_unpack_records(int64_t n, const uint64_t* words, const gw_pack_geom* g, int64_t* key, int64_t* ts,
                      int64_t* value) {
    if (n < 0 || !g || !g->enabled || g->pane <= 0 || (n > 0 && (!words || !key || !ts))) return GW_E_INVALID;
    for (int64_t i = 0; i < n; ++i) {
        int64_t k, t, v;
        unpack_word(*g, words[i], k, t, v);
        key[i] = k;
        ts[i] = t;
        if (value) value[i] = v;
    }
    return GW_OK;
}

int gw_partition_packed_device(int64_t n, const int64_t* d_key, const int64_t* d_ts, const int64_t* d_value,
                               int32_t max_p, int32_t p, const gw_pack_geom* g, uint64_t* d_packed_out,
                               int64_t* d_key_out, int64_t* d_ts_out, int64_t* d_value_out, int64_t* d_counts,
                               void* d_scratch, void* stream) {
    if (n < 0 || max_p <= 0 || p <= 0 || p > max_p || p > 128 || !g || !g->enabled || g->pane <= 0 || !d_counts)
        return GW_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_counts, 0, (size_t)2 * p * 8, s);
        return e == hipSuccess ? GW_OK : GW_E_DEVICE;
    }
    if (!d_key || !d_ts || !d_packed_out || !d_key_out || !d_ts_out || (d_value && !d_value_out) || !d_scratch)
        return GW_E_INVALID;
    hipError_t e = launch_partition(n, d_key, nullptr, d_ts, d_value, max_p, p, d_key_out, d_ts_out, d_value_out,
                                    d_counts, d_scratch, s, nullptr, g, d_packed_out);
    if (e != hipSuccess) { g_create_error = hipGetErrorString(e); return GW_E_DEVICE; }
    return GW_OK;
}

int gw_partition_regions_device(int64_t n, const int64_t* d_key, const int64_t* d_ts, const int64_t* d_value,
                                int32_t max_p, int32_t p, const gw_pack_geom* g, int64_t cap, uint64_t* d_packed_out,
                                int64_t* d_key_out, int64_t* d_ts_out, int64_t* d_value_out, int64_t* d_counts,
                                void* d_scratch, void* stream) {
    const bool packed = g && g->enabled;
    if (n < 0 || max_p <= 0 || p <= 0 || p > max_p || p > kPartRegionMaxOwners || !d_counts || cap < n ||
        (packed && g->pane <= 0))
        return GW_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_counts, 0, (size_t)(packed ? 2 : 1) * p * 8, s);
        return e == hipSuccess ? GW_OK : GW_E_DEVICE;
    }
    if (!d_key || !d_ts || (packed && !d_packed_out) || !d_key_out || !d_ts_out || (d_value && !d_value_out) ||
        !d_scratch)
        return GW_E_INVALID;
    hipError_t e = launch_partition_regions(n, d_key, nullptr, d_ts, d_value, max_p, p, cap, d_key_out, d_ts_out,
                                            d_value_out, nullptr, packed ? g : nullptr, d_packed_out, d_counts,
                                            d_scratch, s);
    if (e != hipSuccess) { g_create_error = hipGetErrorString(e); return GW_E_DEVICE; }
    return GW_OK;
}

int gw_select_lookup_device(int64_t n, const int64_t* d_sel, int64_t sel_value, const int64_t* d_idx,
                            const int64_t* d_dict, int64_t dict_n, const int64_t* d_ts, int64_t* d_key_out,
                            int64_t* d_ts_out, int64_t* n_out, void* stream) {
    if (!n_out || n < 0 || dict_n < 0 || (n > 0 && (!d_sel || !d_idx || !d_ts || !d_key_out || !d_ts_out)) ||
        (dict_n > 0 && !d_dict))
        return GW_E_INVALID;
    *n_out = 0;
    if (n == 0) return GW_OK;
    // scratch per device, grown as needed (every call waits for its launches before returning,
    // so a later call may free it)
    static std::mutex mu;
    static void* scr[64] = {};
    static size_t cap[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return GW_E_DEVICE;
    const size_t need = select_lookup_scratch_bytes(n);
    std::lock_guard<std::mutex> lock(mu);
    if (need > cap[dev]) {
        if (scr[dev]) hipFree(scr[dev]);
        scr[dev] = nullptr;
        cap[dev] = 0;
        if (hipMalloc(&scr[dev], need) != hipSuccess) { g_create_error = "gw_select_lookup_device: scratch"; return GW_E_OOM; }
        cap[dev] = need;
    }
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = launch_select_lookup(n, d_sel, sel_value, d_idx, d_dict, dict_n, d_ts, d_key_out, d_ts_out, scr[dev], s);
    // the total and the range flag sit behind the tile offsets (gw_select.hip)
    const int64_t ntiles = (n + 4095) / 4096;
    const char* tail = (const char*)scr[dev] + ((ntiles * 4 + 15) / 16) * 16 + (size_t)ntiles * 8;
    int64_t hv[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(hv, tail, 16, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { g_create_error = hipGetErrorString(e); return GW_E_DEVICE; }
    if ((int32_t)hv[1]) { g_create_error = "gw_select_lookup_device: index outside the dictionary"; return GW_E_RANGE; }
    *n_out = hv[0];
    return GW_OK;
}

int gw_unpack_device(int64_t n, const uint64_t* d_words, const gw_pack_geom* g, int64_t* d_key, int64_t* d_ts,
                     int64_t* d_value, void* stream) {
    if (n < 0 || !g || !g->enabled || g->pane <= 0 || (n > 0 && (!d_words || !d_key || !d_ts))) return GW_E_INVALID;
    hipError_t e = launch_unpack(n, d_words, *g, d_key, d_ts, d_value, (hipStream_t)stream);
    if (e != hipSuccess) { g_create_error = hipGetErrorString(e); return GW_E_DEVICE; }
    return GW_OK;
}

int gw_partition_device(int64_t n, const int64_t* d_key, const int32_t* d_key_hash, const int64_t* d_ts,
                        const void* d_value, int32_t max_p, int32_t p, int64_t* d_key_out, int64_t* d_ts_out,
                        void* d_value_out, int64_t* d_counts, void* d_scratch, void* stream) {
    if (n < 0 || max_p <= 0 || p <= 0 || p > max_p || p > 256) return GW_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0) {
        hipError_t e = hipMemsetAsync(d_counts, 0, (size_t)p * 8, s);
        return e == hipSuccess ? GW_OK : GW_E_DEVICE;
    }
    hipError_t e = launch_partition(n, d_key, d_key_hash, d_ts, (const int64_t*)d_value, max_p, p, d_key_out,
                                    d_ts_out, (int64_t*)d_value_out, d_counts, d_scratch, s);
    if (e != hipSuccess) { g_create_error = hipGetErrorString(e); return GW_E_DEVICE; }
    return GW_OK;
}

}  // extern "C"
