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
// is an RCCL all-reduce(MIN) of one int64.
#include "gw_kernels.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace gw;

struct gw_exchange {
    ncclComm_t comm = nullptr;
    int32_t nranks = 0, rank = 0, device = 0, max_p = 128;
    void* scratch = nullptr;  // partition scratch
    int64_t scratch_bytes = 0;
    int64_t* part = nullptr;  // partitioned key | ts | value columns, cap records each
    int32_t* part_hash = nullptr;
    int64_t part_cap = 0;
    int64_t* recv[2] = {nullptr, nullptr};  // receive sets used in turn: key | ts | value columns
    int32_t* recv_hash[2] = {nullptr, nullptr};
    int64_t recv_cap[2] = {0, 0};
    int turn = 0;
    // One all-to-all message per peer and batch: (records for it, watermark, column mask).
    // d_msg: [nranks][kMsg] send | [nranks][kMsg] receive; h_msg its pinned copy.
    static constexpr int kMsg = 3;
    int64_t* d_counts = nullptr;  // [nranks] partition counts
    int64_t* d_msg = nullptr;
    int64_t* h_msg = nullptr;
    int64_t* d_wm = nullptr;
    int64_t* h_wm = nullptr;
    std::vector<int64_t> last_send, last_recv;
    std::vector<int64_t> plan[4];  // gw_exchange_plan: send offsets, send counts, receive offsets, receive counts
    // per receive set: the hand-off stream the ingest orders on, and its "reads done" event
    hipStream_t handoff[2] = {nullptr, nullptr};
    hipEvent_t ev_recv[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr};
    bool set_used[2] = {false, false};
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
#define EX_NCCL(x)                                                                           \
    do {                                                                                     \
        ncclResult_t r_ = (x);                                                               \
        if (r_ != ncclSuccess) return ex_fail(ex, GW_E_DEVICE, std::string(#x ": ") + ncclGetErrorString(r_)); \
    } while (0)

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
    ex->device = device;
    ex->max_p = max_parallelism;
    auto bail = [&](int rc) { gw_exchange_destroy(ex); return rc; };
    if (hipSetDevice(device) != hipSuccess) return bail(GW_E_DEVICE);
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&ex->comm, nranks, u, rank) != ncclSuccess) return bail(GW_E_DEVICE);
    const size_t words = (size_t)nranks * (1 + 2 * gw_exchange::kMsg) + 2;
    if (hipMalloc((void**)&ex->d_counts, words * 8) != hipSuccess) return bail(GW_E_OOM);
    if (hipHostMalloc((void**)&ex->h_msg, (size_t)(2 * gw_exchange::kMsg * nranks + 2) * 8, hipHostMallocDefault) !=
        hipSuccess)
        return bail(GW_E_OOM);
    ex->d_msg = ex->d_counts + nranks;
    ex->d_wm = ex->d_msg + 2 * gw_exchange::kMsg * nranks;
    ex->h_wm = ex->h_msg + 2 * gw_exchange::kMsg * nranks;
    for (int q = 0; q < 2; ++q) {
        if (hipStreamCreateWithFlags(&ex->handoff[q], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ex->ev_recv[q], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ex->ev_free[q], hipEventDisableTiming) != hipSuccess)
            return bail(GW_E_DEVICE);
    }
    ex->last_send.assign(nranks, 0);
    ex->last_recv.assign(nranks, 0);
    for (auto& v : ex->plan) v.assign(nranks, 0);
    *out = ex;
    return GW_OK;
}

void gw_exchange_destroy(gw_exchange* ex) {
    if (!ex) return;
    hipDeviceSynchronize();
    if (ex->comm) ncclCommDestroy(ex->comm);
    hipFree(ex->scratch);
    hipFree(ex->part);
    hipFree(ex->part_hash);
    for (int q = 0; q < 2; ++q) { hipFree(ex->recv[q]); hipFree(ex->recv_hash[q]); }
    hipFree(ex->d_counts);
    hipHostFree(ex->h_msg);
    for (int q = 0; q < 2; ++q) {
        if (ex->handoff[q]) hipStreamDestroy(ex->handoff[q]);
        if (ex->ev_recv[q]) hipEventDestroy(ex->ev_recv[q]);
        if (ex->ev_free[q]) hipEventDestroy(ex->ev_free[q]);
    }
    delete ex;
}

const char* gw_exchange_last_error(const gw_exchange* ex) { return ex ? ex->err.c_str() : ""; }

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
        if (s < 0 || r < 0) return GW_E_INVALID;
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

int gw_exchange_batch(gw_exchange* ex, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                      const int64_t* d_ts, const int64_t* d_value, int64_t wm, int64_t* n_out,
                      const int64_t** d_key_out, const int32_t** d_key_hash_out, const int64_t** d_ts_out,
                      const int64_t** d_value_out, int64_t* wm_out, void** ingest_stream, void* stream) {
    if (!ex || n < 0 || !n_out || !d_key_out || !d_ts_out || (n > 0 && (!d_key || !d_ts))) return GW_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    const int P = ex->nranks;
    constexpr int M = gw_exchange::kMsg;
    // 1. stable device partition by owner subtask
    if (n > ex->part_cap) {
        EX_HIP(hipStreamSynchronize(s));
        hipFree(ex->part);
        hipFree(ex->part_hash);
        ex->part = nullptr;
        ex->part_hash = nullptr;
        const int64_t c = n + n / 4 + 1024;
        EX_HIP(hipMalloc((void**)&ex->part, (size_t)c * 3 * 8));
        EX_HIP(hipMalloc((void**)&ex->part_hash, (size_t)c * 4));
        ex->part_cap = c;
    }
    const int64_t need = partition_scratch_bytes(std::max<int64_t>(n, 1), P);
    if (need > ex->scratch_bytes) {
        EX_HIP(hipStreamSynchronize(s));
        hipFree(ex->scratch);
        ex->scratch = nullptr;
        EX_HIP(hipMalloc(&ex->scratch, (size_t)need));
        ex->scratch_bytes = need;
    }
    int64_t* pk = ex->part;
    int64_t* pt = pk + ex->part_cap;
    int64_t* pv = pt + ex->part_cap;
    if (n > 0) {
        EX_HIP(launch_partition(n, d_key, d_key_hash, d_ts, d_value, ex->max_p, P, pk, pt, d_value ? pv : nullptr,
                                ex->d_counts, ex->scratch, s, d_key_hash ? ex->part_hash : nullptr));
    } else {
        EX_HIP(hipMemsetAsync(ex->d_counts, 0, (size_t)P * 8, s));
    }
    // 2. one message per peer: (count, watermark, columns); all-to-all, then one host wait
    const int64_t cols_mask = (d_value ? 1 : 0) | (d_key_hash ? 2 : 0);
    EX_HIP(launch_exchange_message(ex->d_counts, P, wm, cols_mask, ex->d_msg, s));
    EX_NCCL(ncclAllToAll(ex->d_msg, ex->d_msg + M * P, M, ncclInt64, ex->comm, s));
    EX_HIP(hipMemcpyAsync(ex->h_msg, ex->d_msg, (size_t)2 * M * P * 8, hipMemcpyDeviceToHost, s));
    EX_HIP(hipStreamSynchronize(s));
    const int64_t* sm = ex->h_msg;
    const int64_t* rm = ex->h_msg + M * P;
    std::vector<int64_t>& so = ex->plan[0];
    std::vector<int64_t>& sc = ex->plan[1];
    std::vector<int64_t>& ro = ex->plan[2];
    std::vector<int64_t>& rc = ex->plan[3];
    int64_t total = 0, wmin = wm;
    // every rank sees every rank's mask: all of them fail here together, before any send
    if (gw_exchange_plan(P, sm, rm, cols_mask, wm, so.data(), sc.data(), ro.data(), rc.data(), &total, &wmin))
        return ex_fail(ex, GW_E_INVALID, "gw_exchange_batch: ranks pass different columns");
    ex->last_send = sc;
    ex->last_recv = rc;
    // 3. this turn's receive set: free once the ingest two batches ago has read it
    const int u = ex->turn;
    ex->turn ^= 1;
    if (ex->set_used[u]) {  // everything queued on its hand-off stream so far: the ingest's reads
        EX_HIP(hipEventRecord(ex->ev_free[u], ex->handoff[u]));
        EX_HIP(hipStreamWaitEvent(s, ex->ev_free[u], 0));
    }
    if (total > ex->recv_cap[u]) {
        EX_HIP(hipStreamSynchronize(s));
        hipFree(ex->recv[u]);
        hipFree(ex->recv_hash[u]);
        ex->recv[u] = nullptr;
        ex->recv_hash[u] = nullptr;
        const int64_t c = total + total / 4 + 1024;
        EX_HIP(hipMalloc((void**)&ex->recv[u], (size_t)c * 3 * 8));
        EX_HIP(hipMalloc((void**)&ex->recv_hash[u], (size_t)c * 4));
        ex->recv_cap[u] = c;
    }
    int64_t* rk = ex->recv[u];
    int64_t* rt = rk + ex->recv_cap[u];
    int64_t* rv = rt + ex->recv_cap[u];
    int32_t* rh = ex->recv_hash[u];
    // 4. columns: grouped point-to-point send / receive per peer (the group is always closed)
    struct Col { const void* src; void* dst; ncclDataType_t t; size_t w; };
    const Col cols[4] = {{pk, rk, ncclInt64, 8},
                         {pt, rt, ncclInt64, 8},
                         {d_value ? pv : nullptr, rv, ncclInt64, 8},
                         {d_key_hash ? ex->part_hash : nullptr, rh, ncclInt32, 4}};
    EX_NCCL(ncclGroupStart());
    ncclResult_t r = ncclSuccess;
    for (const Col& c : cols) {
        if (!c.src) continue;
        for (int q = 0; q < P && r == ncclSuccess; ++q) {
            if (sc[q]) r = ncclSend((const char*)c.src + so[q] * c.w, (size_t)sc[q], c.t, q, ex->comm, s);
            if (r == ncclSuccess && rc[q]) r = ncclRecv((char*)c.dst + ro[q] * c.w, (size_t)rc[q], c.t, q, ex->comm, s);
        }
    }
    const ncclResult_t re = ncclGroupEnd();
    if (r != ncclSuccess) return ex_fail(ex, GW_E_DEVICE, std::string("ncclSend/ncclRecv: ") + ncclGetErrorString(r));
    if (re != ncclSuccess) return ex_fail(ex, GW_E_DEVICE, std::string("ncclGroupEnd: ") + ncclGetErrorString(re));
    // 5. hand-off: the ingest of this set orders after the receives on handoff[u] (and makes
    // handoff[u] wait for its reads); the exchange that reuses the set waits for handoff[u]
    EX_HIP(hipEventRecord(ex->ev_recv[u], s));
    EX_HIP(hipStreamWaitEvent(ex->handoff[u], ex->ev_recv[u], 0));
    ex->set_used[u] = true;
    *n_out = total;
    *d_key_out = rk;
    *d_ts_out = rt;
    if (d_value_out) *d_value_out = d_value ? rv : nullptr;
    if (d_key_hash_out) *d_key_hash_out = d_key_hash ? rh : nullptr;
    if (wm_out) *wm_out = wmin;
    if (ingest_stream) *ingest_stream = (void*)ex->handoff[u];
    return GW_OK;
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
    hipStream_t s = (hipStream_t)stream;
    *ex->h_wm = wm;
    EX_HIP(hipMemcpyAsync(ex->d_wm, ex->h_wm, 8, hipMemcpyHostToDevice, s));
    EX_NCCL(ncclAllReduce(ex->d_wm, ex->d_wm, 1, ncclInt64, ncclMin, ex->comm, s));
    EX_HIP(hipMemcpyAsync(ex->h_wm, ex->d_wm, 8, hipMemcpyDeviceToHost, s));
    EX_HIP(hipStreamSynchronize(s));
    *out = *ex->h_wm;
    return GW_OK;
}

}  // extern "C"
