// gw_exchange.cpp — the keyBy exchange of one watermark batch between the GPUs of a node
// (include/gpuwin.h, gw_exchange_*), native to libgpuwin so the JVM side drives it
// through the C ABI like the window operator itself.
//
// Reference path replaced: KeyGroupStreamPartitioner.selectChannel (flink-runtime/.../
// streaming/runtime/partitioner/KeyGroupStreamPartitioner.java:55-64) picks the owner
// subtask of every record; RecordWriter (RR/io/network/api/writer/RecordWriter.java:
// 104-110) serializes it into that channel's network buffers; Netty ships them.  Here a
// batch is partitioned on the device (launch_partition: stable, grouped by owner), the
// per-owner counts go through one RCCL all-to-all, and every column moves as one grouped
// ncclSend / ncclRecv per peer (xGMI point-to-point links; no host copy of the records).
// The watermark combine (StatusWatermarkValve.inputWatermark, min over input channels)
// rides the count all-to-all.
//
// Packing (gw_exchange_enable_packing): a record that fits travels as one 8-byte word
// (gw_common.h pack_word: key, value and its pane relative to the watermark before the batch)
// instead of 24 B; the partition sorts each destination's records into (packed, other), both
// go out per peer, and the receiver unpacks the words behind the other records.  The base
// pane comes from the previous batch's combined watermark, which every rank knows alike.
#include "gw_kernels.h"
#include "gw_wait.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace gw;

struct gw_exchange {
    ncclComm_t comm = nullptr;
    int32_t nranks = 0, rank = 0, device = 0, max_p = 128;
    bool no_regions = false;
    // packed batches: region places by atomics, not in arrival order (k_part_regions unstable;
    // GW_PART_STABLE=1 keeps the look-back for every batch)
    bool stable_order = false;
    int part_turn = 0;  // status half of the next region partition  // GW_PART_REGIONS=0: the three-pass contiguous partition (A/B)
    void* scratch = nullptr;  // partition scratch (used only inside a partition launch: shared)
    int64_t scratch_bytes = 0;
    // Two partition sets, so batch b + 1 can be partitioned and its counts exchanged
    // (gw_exchange_begin) before batch b's columns are sent (gw_exchange_finish).
    struct PartSet {
        int64_t* part = nullptr;  // partitioned key | ts | value columns, cap records each
        int32_t* part_hash = nullptr;
        uint64_t* part_packed = nullptr;  // packed words (partition numbering), cap records
        int64_t part_cap = 0;
        int64_t part_regions = 0;  // regions the buffers were allocated for (1: contiguous)
        int64_t* d_counts = nullptr;  // [2 nranks] partition counts (packing: packed, other per peer)
        int64_t* d_msg = nullptr;     // [nranks][kMsg] send | [nranks][kMsg] receive
        int64_t* h_msg = nullptr;     // its pinned copy
        hipEvent_t ev_msg = nullptr;  // after the copy
        // the begun batch
        int64_t n = 0, wm = 0, cols_mask = 0;
        bool regions = false, packed = false, has_value = false, has_hash = false;
        gw_pack_geom g{};
        hipStream_t stream = nullptr;
    } ps[2];
    int64_t begun = 0, finished = 0;  // batches begun / finished (set of batch i: i & 1)
    // Receive sets used in turn (key | ts | value columns, key hashes, packed words).  Three, so
    // batch b's receives wait only for the ingest of batch b - 3 to have read its set: with two,
    // the exchange stream waited on the operator's pass 1 of batch b - 2, which itself runs
    // beside the exchange's partition of a later batch (measured: ~50 us per batch of the
    // exchange stream idling on that cross-stream event, profiles/r6/exchange/).  Finishing
    // batches further ahead of the ingest (bench.py --exchange-ahead 2, or from a host thread of
    // its own with four sets) measured no faster: the partition then runs beside the flush and
    // both slow down (profiles/r6/exchange/driver/).
    static constexpr int kSets = GW_EXCHANGE_RECV_SETS;
    int64_t* recv[kSets] = {};
    int32_t* recv_hash[kSets] = {};
    uint64_t* recv_packed[kSets] = {};
    int64_t recv_cap[kSets] = {};
    int turn = 0;
    // packing (gw_exchange_enable_packing): window geometry and the last combined watermark
    bool pack_on = false, pack_values = false;
    int64_t pack_size = 0, pack_slide = 0, pack_offset = 0;
    int64_t last_wm = INT64_MIN;
    int64_t last_packed = 0;
    bool unpack = true;                    // false: the words stay packed (gw_exchange_last_words)
    const uint64_t* last_words = nullptr;
    gw_pack_geom last_geom{};
    // One all-to-all message per peer and batch: (records for it, watermark, column mask,
    // packed records), per partition set.
    static constexpr int kMsg = 4;
    int64_t* d_wm = nullptr;
    int64_t* h_wm = nullptr;
    std::vector<int64_t> last_send, last_recv;
    std::vector<int64_t> plan[4];  // gw_exchange_plan: send offsets, send counts, receive offsets, receive counts
    std::vector<int64_t> pplan[4];  // gw_exchange_plan_packed: send packed, receive other / packed offsets, packed
    // per receive set: the hand-off stream the ingest orders on, and its "reads done" event
    hipStream_t handoff[kSets] = {};
    hipEvent_t ev_recv[kSets] = {}, ev_free[kSets] = {};
    bool set_used[kSets] = {};
    // fail fast (gw_wait.h): every host wait is bounded; on expiry or an asynchronous RCCL error
    // the communicator is aborted and every later call fails with GW_E_STATE
    int64_t timeout_ms = 60000;
    bool aborted = false;
    hipStream_t last_stream = nullptr;  // the caller's exchange stream of the last batch
    std::string err;
};

static int ex_fail(gw_exchange* ex, int rc, const std::string& what) {
    if (ex) ex->err = what;
    return rc;
}
#define EX_HIP(x)                                                                            \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) return ex_fail(ex, GW_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)
#define EX_LIVE(ex)                                                                          \
    do {                                                                                     \
        if ((ex)->aborted)                                                                   \
            return ex_fail(ex, GW_E_STATE, "exchange aborted after an earlier failure: " + (ex)->err); \
    } while (0)
#define EX_NCCL(x)                                                                           \
    do {                                                                                     \
        ncclResult_t r_ = (x);                                                               \
        if (r_ != ncclSuccess) return ex_fail(ex, GW_E_DEVICE, std::string(#x ": ") + ncclGetErrorString(r_)); \
    } while (0)

static void ex_abort(gw_exchange* ex) {
    if (ex->aborted) return;
    ex->aborted = true;
    if (ex->comm) {
        (void)ncclCommAbort(ex->comm);  // kernels waiting on a dead peer return; the communicator is gone
        ex->comm = nullptr;
    }
}

// Wait for everything queued on s (a collective and what follows it), bounded: the stream
// completes, or its error, the communicator's asynchronous error or the deadline aborts the
// communicator and fails the call (GW_E_STATE; the JVM side throws and fails the task).
static int ex_wait(gw_exchange* ex, hipStream_t s, const char* what) {
    EX_LIVE(ex);
    hipError_t herr = hipSuccess;
    ncclResult_t aerr = ncclSuccess;
    const WaitResult w = poll_until_done(
        [&] {
            herr = hipStreamQuery(s);
            return herr == hipSuccess ? 0 : herr == hipErrorNotReady ? 1 : 2;
        },
        [&] {
            if (ncclCommGetAsyncError(ex->comm, &aerr) != ncclSuccess) return 1;
            return aerr == ncclSuccess || aerr == ncclInProgress ? 0 : 1;
        },
        steady_now_ns, relax_backoff, ex->timeout_ms * 1000000);
    if (w == WaitResult::kDone) return GW_OK;
    std::string why = std::string(what) + ": ";
    if (w == WaitResult::kStreamError) why += std::string("stream error: ") + hipGetErrorString(herr);
    else if (w == WaitResult::kCommError) why += std::string("RCCL asynchronous error: ") + ncclGetErrorString(aerr);
    else why += "no completion within " + std::to_string(ex->timeout_ms) + " ms (a peer died or diverged)";
    ex_abort(ex);
    return ex_fail(ex, GW_E_STATE, why + "; communicator aborted");
}

// The same for one event (gw_exchange_finish: the count all-to-all's copy to the host).
static int ex_wait_event(gw_exchange* ex, hipEvent_t ev, const char* what) {
    EX_LIVE(ex);
    hipError_t herr = hipSuccess;
    ncclResult_t aerr = ncclSuccess;
    const WaitResult w = poll_until_done(
        [&] {
            herr = hipEventQuery(ev);
            return herr == hipSuccess ? 0 : herr == hipErrorNotReady ? 1 : 2;
        },
        [&] {
            if (ncclCommGetAsyncError(ex->comm, &aerr) != ncclSuccess) return 1;
            return aerr == ncclSuccess || aerr == ncclInProgress ? 0 : 1;
        },
        steady_now_ns, relax_backoff, ex->timeout_ms * 1000000);
    if (w == WaitResult::kDone) return GW_OK;
    std::string why = std::string(what) + ": ";
    if (w == WaitResult::kStreamError) why += std::string("stream error: ") + hipGetErrorString(herr);
    else if (w == WaitResult::kCommError) why += std::string("RCCL asynchronous error: ") + ncclGetErrorString(aerr);
    else why += "no completion within " + std::to_string(ex->timeout_ms) + " ms (a peer died or diverged)";
    ex_abort(ex);
    return ex_fail(ex, GW_E_STATE, why + "; communicator aborted");
}

extern "C" {

int gw_exchange_unique_id(void* id) {
    static_assert(sizeof(ncclUniqueId) == GW_EXCHANGE_ID_BYTES, "ncclUniqueId size");
    if (!id) return GW_E_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return GW_E_DEVICE;
    memcpy(id, &u, sizeof(u));
    return GW_OK;
}

int gw_exchange_create(gw_exchange** out, int32_t nranks, int32_t rank, const void* id, int32_t device,
                       int32_t max_parallelism) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks || max_parallelism < nranks ||
        nranks > 256)
        return GW_E_INVALID;
    *out = nullptr;
    gw_exchange* ex = new gw_exchange();
    ex->nranks = nranks;
    ex->rank = rank;
    if (const char* e = getenv("GW_PART_REGIONS")) ex->no_regions = atoi(e) == 0;
    if (const char* e = getenv("GW_PART_STABLE")) ex->stable_order = atoi(e) != 0;
    ex->device = device;
    ex->max_p = max_parallelism;
    auto bail = [&](int rc) { gw_exchange_destroy(ex); return rc; };
    if (hipSetDevice(device) != hipSuccess) return bail(GW_E_DEVICE);
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&ex->comm, nranks, u, rank) != ncclSuccess) return bail(GW_E_DEVICE);
    const size_t words = (size_t)nranks * (2 + 2 * gw_exchange::kMsg);
    for (auto& q : ex->ps) {
        if (hipMalloc((void**)&q.d_counts, words * 8) != hipSuccess) return bail(GW_E_OOM);
        // the unstable region partition adds into the counts (k_exchange_message zeroes them after)
        if (hipMemset(q.d_counts, 0, words * 8) != hipSuccess) return bail(GW_E_DEVICE);
        if (hipHostMalloc((void**)&q.h_msg, (size_t)(2 * gw_exchange::kMsg * nranks) * 8, hipHostMallocDefault) !=
            hipSuccess)
            return bail(GW_E_OOM);
        q.d_msg = q.d_counts + 2 * nranks;
        if (hipEventCreateWithFlags(&q.ev_msg, hipEventDisableTiming) != hipSuccess) return bail(GW_E_DEVICE);
    }
    if (hipMalloc((void**)&ex->d_wm, 8) != hipSuccess) return bail(GW_E_OOM);
    if (hipHostMalloc((void**)&ex->h_wm, 8, hipHostMallocDefault) != hipSuccess) return bail(GW_E_OOM);
    for (int q = 0; q < gw_exchange::kSets; ++q) {
        if (hipStreamCreateWithFlags(&ex->handoff[q], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ex->ev_recv[q], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ex->ev_free[q], hipEventDisableTiming) != hipSuccess)
            return bail(GW_E_DEVICE);
    }
    ex->last_send.assign(nranks, 0);
    ex->last_recv.assign(nranks, 0);
    for (auto& v : ex->plan) v.assign(nranks, 0);
    for (auto& v : ex->pplan) v.assign(nranks, 0);
    *out = ex;
    return GW_OK;
}

void gw_exchange_destroy(gw_exchange* ex) {
    if (!ex) return;
    // the last batch's collectives may still wait on a peer: bounded, then abort
    if (!ex->aborted && ex->last_stream && ex_wait(ex, ex->last_stream, "gw_exchange_destroy") != GW_OK) {
        // aborted: the kernels that waited on the peer have returned
    }
    for (int q = 0; q < gw_exchange::kSets; ++q)
        if (!ex->aborted && ex->handoff[q]) (void)ex_wait(ex, ex->handoff[q], "gw_exchange_destroy");
    if (!ex->aborted) (void)hipDeviceSynchronize();
    if (ex->comm) ncclCommDestroy(ex->comm);
    hipFree(ex->scratch);
    for (auto& q : ex->ps) {
        hipFree(q.part);
        hipFree(q.part_hash);
        hipFree(q.part_packed);
        hipFree(q.d_counts);
        hipHostFree(q.h_msg);
        if (q.ev_msg) hipEventDestroy(q.ev_msg);
    }
    for (int q = 0; q < gw_exchange::kSets; ++q) { hipFree(ex->recv[q]); hipFree(ex->recv_hash[q]); hipFree(ex->recv_packed[q]); }
    hipFree(ex->d_wm);
    hipHostFree(ex->h_wm);
    for (int q = 0; q < gw_exchange::kSets; ++q) {
        if (ex->handoff[q]) hipStreamDestroy(ex->handoff[q]);
        if (ex->ev_recv[q]) hipEventDestroy(ex->ev_recv[q]);
        if (ex->ev_free[q]) hipEventDestroy(ex->ev_free[q]);
    }
    delete ex;
}

const char* gw_exchange_last_error(const gw_exchange* ex) { return ex ? ex->err.c_str() : ""; }

int gw_exchange_set_timeout(gw_exchange* ex, int64_t timeout_ms) {
    if (!ex || timeout_ms < 0) return GW_E_INVALID;
    ex->timeout_ms = timeout_ms;
    return GW_OK;
}

int gw_exchange_plan(int32_t nranks, const int64_t* sent_msg, const int64_t* recv_msg, int64_t cols_mask, int64_t wm,
                     int64_t* send_off, int64_t* send_cnt, int64_t* recv_off, int64_t* recv_cnt, int64_t* total,
                     int64_t* wm_min) {
    constexpr int M = gw_exchange::kMsg;
    if (nranks < 1 || !sent_msg || !recv_msg || !send_off || !send_cnt || !recv_off || !recv_cnt || !total || !wm_min)
        return GW_E_INVALID;
    int64_t so = 0, ro = 0, wmin = wm;
    bool agree = true;
    for (int q = 0; q < nranks; ++q) {
        const int64_t s = sent_msg[M * q], r = recv_msg[M * q];
        const int64_t sp = sent_msg[M * q + 3], rp = recv_msg[M * q + 3];
        if (s < 0 || r < 0 || sp < 0 || sp > s || rp < 0 || rp > r) return GW_E_INVALID;
        send_off[q] = so;
        send_cnt[q] = s;
        recv_off[q] = ro;
        recv_cnt[q] = r;
        so += s;
        ro += r;
        wmin = std::min(wmin, recv_msg[M * q + 1]);
        agree &= recv_msg[M * q + 2] == cols_mask;
    }
    *total = ro;
    *wm_min = wmin;
    return agree ? GW_OK : GW_E_INVALID;
}

int gw_exchange_plan_packed(int32_t nranks, const int64_t* sent_msg, const int64_t* recv_msg, int64_t* send_packed,
                            int64_t* recv_other_off, int64_t* recv_packed_off, int64_t* recv_packed,
                            int64_t* total_other, int64_t* total_packed) {
    constexpr int M = gw_exchange::kMsg;
    if (nranks < 1 || !sent_msg || !recv_msg || !send_packed || !recv_other_off || !recv_packed_off ||
        !recv_packed || !total_other || !total_packed)
        return GW_E_INVALID;
    int64_t wo = 0, po = 0;
    for (int q = 0; q < nranks; ++q) {
        const int64_t s = sent_msg[M * q], r = recv_msg[M * q];
        const int64_t sp = sent_msg[M * q + 3], rp = recv_msg[M * q + 3];
        if (s < 0 || r < 0 || sp < 0 || sp > s || rp < 0 || rp > r) return GW_E_INVALID;
        send_packed[q] = sp;
        recv_other_off[q] = wo;
        recv_packed_off[q] = po;
        recv_packed[q] = rp;
        wo += r - rp;
        po += rp;
    }
    *total_other = wo;
    *total_packed = po;
    return GW_OK;
}

typedef __int128 i128;
// Region-partition buffers above this fall back to the contiguous layout (36 B x P
// per record of capacity is ~72 GB per rank at 16 ranks and 100M-record batches).
constexpr int64_t kRegionBudget = (int64_t)16 << 30;

// (pane, offset, base pane) of a packing geometry folded to 32 non-zero bits
static uint64_t geom_fold(const gw_pack_geom& g) {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (int64_t v : {g.pane, g.offset, g.base_pane}) {
        h ^= (uint64_t)v;
        h *= 0xbf58476d1ce4e5b9ull;
        h ^= h >> 31;
    }
    return (h >> 32) | 1;
}

static int64_t gcd64(int64_t a, int64_t b) {
    while (b) { const int64_t t = a % b; a = b; b = t; }
    return a;
}

int gw_pack_geom_init(gw_pack_geom* g, int64_t size, int64_t slide, int64_t offset, int64_t watermark) {
    if (!g || size <= 0 || slide <= 0) return GW_E_INVALID;
    *g = gw_pack_geom{};
    if (size < slide || watermark == INT64_MIN) return GW_E_UNSUPPORTED;
    const int64_t pane = gcd64(size, slide);
    __int128 rel = (__int128)watermark - offset;
    __int128 q = rel / pane;
    if (rel % pane < 0) --q;
    if (q > INT64_MAX || q < INT64_MIN) return GW_E_UNSUPPORTED;
    g->pane = pane;
    g->offset = offset;
    g->base_pane = (int64_t)q;
    g->enabled = 1;
    return GW_OK;
}

int gw_exchange_enable_packing(gw_exchange* ex, int64_t size, int64_t slide, int64_t offset, int32_t with_values) {
    if (!ex || size <= 0 || slide <= 0) return GW_E_INVALID;
    if (size < slide) return ex_fail(ex, GW_E_UNSUPPORTED, "packing needs size >= slide");
    if (ex->nranks > 128) return ex_fail(ex, GW_E_UNSUPPORTED, "packing needs <= 128 ranks");
    ex->pack_on = true;
    ex->pack_values = with_values != 0;
    ex->pack_size = size;
    ex->pack_slide = slide;
    ex->pack_offset = offset;
    return GW_OK;
}

int64_t gw_exchange_last_packed(const gw_exchange* ex) { return ex ? ex->last_packed : 0; }

int gw_exchange_set_unpack(gw_exchange* ex, int32_t unpack) {
    if (!ex) return GW_E_INVALID;
    ex->unpack = unpack != 0;
    return GW_OK;
}

int gw_exchange_last_words(const gw_exchange* ex, int64_t* n_words, const uint64_t** d_words, gw_pack_geom* g) {
    if (!ex || !n_words || !d_words) return GW_E_INVALID;
    *n_words = ex->last_words ? ex->last_packed : 0;
    *d_words = ex->last_words;
    if (g) *g = ex->last_geom;
    return GW_OK;
}

int gw_exchange_begin(gw_exchange* ex, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                      const int64_t* d_ts, const int64_t* d_value, int64_t wm, void* stream) {
    if (!ex || n < 0 || (n > 0 && (!d_key || !d_ts))) return GW_E_INVALID;
    EX_LIVE(ex);
    EX_HIP(hipSetDevice(ex->device));  // the calling thread's device (a driver may run the exchange on a thread of its own)
    if (ex->begun - ex->finished >= 2)
        return ex_fail(ex, GW_E_STATE, "gw_exchange_begin: two batches begun and not finished");
    hipStream_t s = (hipStream_t)stream;
    ex->last_stream = s;
    gw_exchange::PartSet& q = ex->ps[ex->begun & 1];
    const int P = ex->nranks;
    constexpr int M = gw_exchange::kMsg;
    // packing this batch: configured, a combined watermark known from a finished batch, no
    // key-hash column, and values only if the caller declared them packable -- the same on
    // every rank (the message check in gw_exchange_finish fails every rank otherwise)
    gw_pack_geom g{};
    if (ex->pack_on && !d_key_hash && (!d_value || ex->pack_values))
        (void)gw_pack_geom_init(&g, ex->pack_size, ex->pack_slide, ex->pack_offset, ex->last_wm);
    const bool packed = g.enabled != 0;
    // 1. stable device partition by owner (packing: by owner, then packed / not).  Up to
    // kPartRegionMaxOwners ranks into one region per owner (single pass, buffers P times the
    // batch: 24 B of columns + 8 B of words per record and region, + 4 B with a key-hash
    // column); past kRegionBudget, or beyond 16 ranks, the contiguous three-pass layout,
    // whose buffers hold the batch once.  The choice is local to the rank.
    const int64_t want_cap = std::max(n + n / 4 + 1024, q.part_cap);
    const bool regions = P <= kPartRegionMaxOwners && !ex->no_regions &&
                         (i128)want_cap * P * (32 + (d_key_hash ? 4 : 0)) <= (i128)kRegionBudget;
    const int64_t R = regions ? P : 1;
    if (n > q.part_cap || R != q.part_regions) {
        const int rc_w = ex_wait(ex, s, "partition buffer");  // this set's last sends read them
        if (rc_w != GW_OK) return rc_w;
        hipFree(q.part);
        hipFree(q.part_hash);
        hipFree(q.part_packed);
        q.part = nullptr;
        q.part_hash = nullptr;
        q.part_packed = nullptr;
        EX_HIP(hipMalloc((void**)&q.part, (size_t)want_cap * R * 3 * 8));
        q.part_cap = want_cap;
        q.part_regions = R;
    }
    if (d_key_hash && !q.part_hash) EX_HIP(hipMalloc((void**)&q.part_hash, (size_t)q.part_cap * R * 4));
    if (packed && !q.part_packed) EX_HIP(hipMalloc((void**)&q.part_packed, (size_t)q.part_cap * R * 8));
    const int64_t need = regions ? partition_regions_scratch_bytes(q.part_cap, 2 * P)
                                 : partition_scratch_bytes(std::max<int64_t>(n, 1), 2 * P);
    if (need > ex->scratch_bytes) {
        const int rc_w = ex_wait(ex, s, "partition scratch");
        if (rc_w != GW_OK) return rc_w;
        hipFree(ex->scratch);
        ex->scratch = nullptr;
        EX_HIP(hipMalloc(&ex->scratch, (size_t)need));
        ex->scratch_bytes = need;
        EX_HIP(hipMemsetAsync(ex->scratch, 0, (size_t)need, s));  // both status halves start zeroed
        ex->part_turn = 0;
    }
    const int64_t col = q.part_cap * R;  // one column of the partition buffer
    int64_t* pk = q.part;
    int64_t* pt = pk + col;
    int64_t* pv = pt + col;
    if (n > 0 && regions) {
        EX_HIP(launch_partition_regions(n, d_key, d_key_hash, d_ts, d_value, ex->max_p, P, q.part_cap, pk, pt,
                                        d_value ? pv : nullptr, d_key_hash ? q.part_hash : nullptr,
                                        packed ? &g : nullptr, q.part_packed, q.d_counts, ex->scratch, s,
                                        ex->part_turn, 2 * P, packed && !ex->stable_order ? 1 : 0));
        ex->part_turn ^= 1;
    } else if (n > 0) {
        EX_HIP(launch_partition(n, d_key, d_key_hash, d_ts, d_value, ex->max_p, P, pk, pt, d_value ? pv : nullptr,
                                q.d_counts, ex->scratch, s, d_key_hash ? q.part_hash : nullptr,
                                packed ? &g : nullptr, q.part_packed));
    } else {
        EX_HIP(hipMemsetAsync(q.d_counts, 0, (size_t)2 * P * 8, s));
    }
    // 2. one message per peer: (records, watermark, columns, packed records); the all-to-all
    // and its copy to the host are queued here, the host reads them in gw_exchange_finish.
    // The column mask also carries the packing geometry (pane, offset, base pane) folded to 32
    // bits: ranks packing against different windows fail together instead of decoding each
    // other's words with the wrong panes.
    q.cols_mask = (d_value ? 1 : 0) | (d_key_hash ? 2 : 0) | (packed ? 4 : 0) |
                  (packed ? (int64_t)(geom_fold(g) << 32) : 0);
    EX_HIP(launch_exchange_message(q.d_counts, P, wm, q.cols_mask, packed ? 1 : 0, q.d_msg, s));
    EX_NCCL(ncclAllToAll(q.d_msg, q.d_msg + M * P, M, ncclInt64, ex->comm, s));
    EX_HIP(hipMemcpyAsync(q.h_msg, q.d_msg, (size_t)2 * M * P * 8, hipMemcpyDeviceToHost, s));
    EX_HIP(hipEventRecord(q.ev_msg, s));
    q.n = n;
    q.wm = wm;
    q.regions = regions;
    q.packed = packed;
    q.g = g;
    q.has_value = d_value != nullptr;
    q.has_hash = d_key_hash != nullptr;
    q.stream = s;
    ex->begun++;
    return GW_OK;
}

int gw_exchange_finish(gw_exchange* ex, int64_t* n_out, const int64_t** d_key_out, const int32_t** d_key_hash_out,
                       const int64_t** d_ts_out, const int64_t** d_value_out, int64_t* wm_out, void** ingest_stream,
                       void* stream) {
    if (!ex || !n_out || !d_key_out || !d_ts_out) return GW_E_INVALID;
    EX_LIVE(ex);
    EX_HIP(hipSetDevice(ex->device));
    if (ex->finished == ex->begun) return ex_fail(ex, GW_E_STATE, "gw_exchange_finish: no batch begun");
    hipStream_t s = (hipStream_t)stream;
    gw_exchange::PartSet& q = ex->ps[ex->finished & 1];
    if (s != q.stream) return ex_fail(ex, GW_E_INVALID, "gw_exchange_finish: not the stream the batch began on");
    const int P = ex->nranks;
    constexpr int M = gw_exchange::kMsg;
    // the host's one wait per batch: this batch's count all-to-all (the next batch's partition,
    // begun already, keeps the stream busy meanwhile)
    {
        const int rc_w = ex_wait_event(ex, q.ev_msg, "gw_exchange_finish: count all-to-all");
        if (rc_w != GW_OK) return rc_w;
    }
    const bool packed = q.packed, regions = q.regions;
    const gw_pack_geom g = q.g;
    const int64_t* sm = q.h_msg;
    const int64_t* rm = q.h_msg + M * P;
    std::vector<int64_t>& so = ex->plan[0];
    std::vector<int64_t>& sc = ex->plan[1];
    std::vector<int64_t>& ro = ex->plan[2];
    std::vector<int64_t>& rc = ex->plan[3];
    std::vector<int64_t>& sp = ex->pplan[0];
    std::vector<int64_t>& rwo = ex->pplan[1];
    std::vector<int64_t>& rpo = ex->pplan[2];
    std::vector<int64_t>& rp = ex->pplan[3];
    int64_t total = 0, wmin = q.wm, tw = 0, tp = 0;
    // every rank sees every rank's mask: all of them fail here together, before any send
    if (gw_exchange_plan(P, sm, rm, q.cols_mask, q.wm, so.data(), sc.data(), ro.data(), rc.data(), &total, &wmin)) {
        ex->finished++;
        return ex_fail(ex, GW_E_INVALID, "gw_exchange_batch: ranks pass different columns or packing geometry");
    }
    if (gw_exchange_plan_packed(P, sm, rm, sp.data(), rwo.data(), rpo.data(), rp.data(), &tw, &tp)) {
        ex->finished++;
        return ex_fail(ex, GW_E_INVALID, "gw_exchange_batch: bad packed counts");
    }
    ex->finished++;
    ex->last_send = sc;
    ex->last_recv = rc;
    ex->last_packed = tp;
    ex->last_wm = wmin;  // the base pane of the batches begun from now on
    // 3. this turn's receive set: free once the ingest three batches ago has read it
    const int u = ex->turn;
    ex->turn = (ex->turn + 1) % gw_exchange::kSets;
    if (ex->set_used[u]) {  // everything queued on its hand-off stream so far: the ingest's reads
        EX_HIP(hipEventRecord(ex->ev_free[u], ex->handoff[u]));
        EX_HIP(hipStreamWaitEvent(s, ex->ev_free[u], 0));
    }
    if (total > ex->recv_cap[u]) {
        {
            const int rc_w = ex_wait(ex, s, "receive buffer");
            if (rc_w != GW_OK) return rc_w;
        }
        hipFree(ex->recv[u]);
        hipFree(ex->recv_hash[u]);
        hipFree(ex->recv_packed[u]);
        ex->recv[u] = nullptr;
        ex->recv_hash[u] = nullptr;
        ex->recv_packed[u] = nullptr;
        const int64_t c = total + total / 4 + 1024;
        EX_HIP(hipMalloc((void**)&ex->recv[u], (size_t)c * 3 * 8));
        ex->recv_cap[u] = c;
    }
    if (q.has_hash && !ex->recv_hash[u]) EX_HIP(hipMalloc((void**)&ex->recv_hash[u], (size_t)ex->recv_cap[u] * 4));
    if (packed && !ex->recv_packed[u]) EX_HIP(hipMalloc((void**)&ex->recv_packed[u], (size_t)ex->recv_cap[u] * 8));
    int64_t* rk = ex->recv[u];
    int64_t* rt = rk + ex->recv_cap[u];
    int64_t* rv = rt + ex->recv_cap[u];
    int32_t* rh = ex->recv_hash[u];
    const int64_t col = q.part_cap * q.part_regions;
    int64_t* pk = q.part;
    int64_t* pt = pk + col;
    int64_t* pv = pt + col;
    // 4. grouped point-to-point send / receive per peer (the group is always closed): per
    // peer its packed words, then each column of its other records, which land behind the
    // other peers' other records in rank order; the unpacked words follow them all
    struct Col { const void* src; void* dst; ncclDataType_t t; size_t w; };
    const Col cols[4] = {{pk, rk, ncclInt64, 8},
                         {pt, rt, ncclInt64, 8},
                         {q.has_value ? pv : nullptr, rv, ncclInt64, 8},
                         {q.has_hash ? q.part_hash : nullptr, rh, ncclInt32, 4}};
    // The rank's own share does not leave the device: a device-to-device copy on the same
    // stream (the copy engine path runs at HBM speed; RCCL's send/receive to self ran its
    // copy on a few channels, ~1 TB/s), queued after the group so it overlaps nothing it must
    // not.  At P ranks it is 1/P of the records.
    const int me = ex->rank;
    // where peer q's packed words / other records start in the partition buffers
    auto pw_off = [&](int r) -> int64_t { return regions ? r * q.part_cap : so[r]; };
    auto pc_off = [&](int r) -> int64_t { return regions ? r * q.part_cap : so[r] + sp[r]; };
    EX_NCCL(ncclGroupStart());
    ncclResult_t r = ncclSuccess;
    for (int pe = 0; pe < P && r == ncclSuccess && packed; ++pe) {
        if (pe == me) continue;
        if (sp[pe]) r = ncclSend(q.part_packed + pw_off(pe), (size_t)sp[pe], ncclUint64, pe, ex->comm, s);
        if (r == ncclSuccess && rp[pe]) r = ncclRecv(ex->recv_packed[u] + rpo[pe], (size_t)rp[pe], ncclUint64, pe, ex->comm, s);
    }
    for (const Col& c : cols) {
        if (!c.src) continue;
        for (int pe = 0; pe < P && r == ncclSuccess; ++pe) {
            if (pe == me) continue;
            const int64_t ns = sc[pe] - sp[pe], nr = rc[pe] - rp[pe];
            if (ns) r = ncclSend((const char*)c.src + pc_off(pe) * c.w, (size_t)ns, c.t, pe, ex->comm, s);
            if (r == ncclSuccess && nr) r = ncclRecv((char*)c.dst + rwo[pe] * c.w, (size_t)nr, c.t, pe, ex->comm, s);
        }
    }
    const ncclResult_t re = ncclGroupEnd();
    if (r != ncclSuccess) return ex_fail(ex, GW_E_DEVICE, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
    if (re != ncclSuccess) return ex_fail(ex, GW_E_DEVICE, std::string("ncclGroupEnd: ") + ncclGetErrorString(re));
    if (packed && sp[me])  // send count = receive count for the rank itself
        EX_HIP(hipMemcpyAsync(ex->recv_packed[u] + rpo[me], q.part_packed + pw_off(me), (size_t)sp[me] * 8,
                              hipMemcpyDeviceToDevice, s));
    for (const Col& c : cols) {
        const int64_t ns = sc[me] - sp[me];
        if (c.src && ns)
            EX_HIP(hipMemcpyAsync((char*)c.dst + rwo[me] * c.w, (const char*)c.src + pc_off(me) * c.w,
                                  (size_t)ns * c.w, hipMemcpyDeviceToDevice, s));
    }
    ex->last_words = nullptr;
    ex->last_geom = g;
    if (packed && tp > 0) {
        if (ex->unpack)
            EX_HIP(launch_unpack(tp, ex->recv_packed[u], g, rk + tw, rt + tw, q.has_value ? rv + tw : nullptr, s));
        else
            ex->last_words = ex->recv_packed[u];
    }
    const int64_t n_cols = (packed && !ex->unpack) ? tw : total;  // records in the columns
    // 5. hand-off: the ingest of this set orders after the receives on handoff[u] (and makes
    // handoff[u] wait for its reads); the exchange that reuses the set waits for handoff[u]
    EX_HIP(hipEventRecord(ex->ev_recv[u], s));
    EX_HIP(hipStreamWaitEvent(ex->handoff[u], ex->ev_recv[u], 0));
    ex->set_used[u] = true;
    *n_out = n_cols;
    *d_key_out = rk;
    *d_ts_out = rt;
    if (d_value_out) *d_value_out = q.has_value ? rv : nullptr;
    if (d_key_hash_out) *d_key_hash_out = q.has_hash ? rh : nullptr;
    if (wm_out) *wm_out = wmin;
    if (ingest_stream) *ingest_stream = (void*)ex->handoff[u];
    return GW_OK;
}

int gw_exchange_batch(gw_exchange* ex, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                      const int64_t* d_ts, const int64_t* d_value, int64_t wm, int64_t* n_out,
                      const int64_t** d_key_out, const int32_t** d_key_hash_out, const int64_t** d_ts_out,
                      const int64_t** d_value_out, int64_t* wm_out, void** ingest_stream, void* stream) {
    if (!ex || n < 0 || !n_out || !d_key_out || !d_ts_out || (n > 0 && (!d_key || !d_ts))) return GW_E_INVALID;
    if (ex->begun != ex->finished)
        return ex_fail(ex, GW_E_STATE, "gw_exchange_batch with a batch begun: finish it first");
    const int rc = gw_exchange_begin(ex, n, d_key, d_key_hash, d_ts, d_value, wm, stream);
    if (rc != GW_OK) return rc;
    return gw_exchange_finish(ex, n_out, d_key_out, d_key_hash_out, d_ts_out, d_value_out, wm_out, ingest_stream,
                              stream);
}

int gw_exchange_counts(const gw_exchange* ex, int64_t* send, int64_t* recv) {
    if (!ex) return GW_E_INVALID;
    for (int q = 0; q < ex->nranks; ++q) {
        if (send) send[q] = ex->last_send[q];
        if (recv) recv[q] = ex->last_recv[q];
    }
    return GW_OK;
}

int gw_exchange_min_watermark(gw_exchange* ex, int64_t wm, int64_t* out, void* stream) {
    if (!ex || !out) return GW_E_INVALID;
    EX_LIVE(ex);
    hipStream_t s = (hipStream_t)stream;
    ex->last_stream = s;
    *ex->h_wm = wm;
    EX_HIP(hipMemcpyAsync(ex->d_wm, ex->h_wm, 8, hipMemcpyHostToDevice, s));
    EX_NCCL(ncclAllReduce(ex->d_wm, ex->d_wm, 1, ncclInt64, ncclMin, ex->comm, s));
    EX_HIP(hipMemcpyAsync(ex->h_wm, ex->d_wm, 8, hipMemcpyDeviceToHost, s));
    {
        const int rc_w = ex_wait(ex, s, "gw_exchange_min_watermark");
        if (rc_w != GW_OK) return rc_w;
    }
    *out = *ex->h_wm;
    return GW_OK;
}

}  // extern "C"
