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
    int64_t* d_counts = nullptr;  // [2][nranks]: send counts | receive counts
    int64_t* h_counts = nullptr;  // pinned copy
    int64_t* d_wm = nullptr;
    int64_t* h_wm = nullptr;
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
    if (hipMalloc((void**)&ex->d_counts, (size_t)2 * nranks * 8 + 16) != hipSuccess) return bail(GW_E_OOM);
    if (hipHostMalloc((void**)&ex->h_counts, (size_t)2 * nranks * 8 + 16, hipHostMallocDefault) != hipSuccess)
        return bail(GW_E_OOM);
    ex->d_wm = ex->d_counts + 2 * nranks;
    ex->h_wm = ex->h_counts + 2 * nranks;
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
    hipHostFree(ex->h_counts);
    delete ex;
}

const char* gw_exchange_last_error(const gw_exchange* ex) { return ex ? ex->err.c_str() : ""; }

int gw_exchange_batch(gw_exchange* ex, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                      const int64_t* d_ts, const int64_t* d_value, int64_t* n_out, const int64_t** d_key_out,
                      const int32_t** d_key_hash_out, const int64_t** d_ts_out, const int64_t** d_value_out,
                      void* stream) {
    if (!ex || n < 0 || !n_out || !d_key_out || !d_ts_out || (n > 0 && (!d_key || !d_ts))) return GW_E_INVALID;
    hipStream_t s = (hipStream_t)stream;
    const int P = ex->nranks;
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
    // 2. counts: all-to-all of one int64 per peer, then to the host (the receive sizes)
    EX_NCCL(ncclAllToAll(ex->d_counts, ex->d_counts + P, 1, ncclInt64, ex->comm, s));
    EX_HIP(hipMemcpyAsync(ex->h_counts, ex->d_counts, (size_t)2 * P * 8, hipMemcpyDeviceToHost, s));
    EX_HIP(hipStreamSynchronize(s));
    const int64_t* sc = ex->h_counts;
    const int64_t* rc = ex->h_counts + P;
    int64_t total = 0;
    for (int q = 0; q < P; ++q) total += rc[q];
    // 3. this turn's receive set, grown to the batch (the stream is idle here)
    const int u = ex->turn;
    ex->turn ^= 1;
    if (total > ex->recv_cap[u]) {
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
    // 4. columns: grouped point-to-point send / receive per peer
    struct Col { const void* src; void* dst; ncclDataType_t t; size_t w; };
    const Col cols[4] = {{pk, rk, ncclInt64, 8},
                         {pt, rt, ncclInt64, 8},
                         {d_value ? pv : nullptr, rv, ncclInt64, 8},
                         {d_key_hash ? ex->part_hash : nullptr, rh, ncclInt32, 4}};
    EX_NCCL(ncclGroupStart());
    for (const Col& c : cols) {
        if (!c.src) continue;
        int64_t so = 0, ro = 0;
        for (int q = 0; q < P; ++q) {
            if (sc[q]) EX_NCCL(ncclSend((const char*)c.src + so * c.w, (size_t)sc[q], c.t, q, ex->comm, s));
            if (rc[q]) EX_NCCL(ncclRecv((char*)c.dst + ro * c.w, (size_t)rc[q], c.t, q, ex->comm, s));
            so += sc[q];
            ro += rc[q];
        }
    }
    EX_NCCL(ncclGroupEnd());
    *n_out = total;
    *d_key_out = rk;
    *d_ts_out = rt;
    if (d_value_out) *d_value_out = d_value ? rv : nullptr;
    if (d_key_hash_out) *d_key_hash_out = d_key_hash ? rh : nullptr;
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
