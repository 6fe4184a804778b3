// gw_netbuf.hip — network-buffer ingest: decode one input channel's serialized stream
// elements into the operator's key / timestamp / value columns on the GPU.
//
// The bytes are what a keyBy channel delivers: per element a 4-byte big-endian length
// (RecordWriter.serializeRecord, flink-runtime/src/main/java/org/apache/flink/runtime/io/
// network/api/writer/RecordWriter.java:144-156; read back by NonSpanningWrapper.readInt
// :142-144), then StreamElementSerializer's tag and body (RS/runtime/streamrecord/
// StreamElementSerializer.java:163-225), the record value written by TupleSerializer
// (flink-core/.../api/java/typeutils/runtime/TupleSerializer.java:135-144).
//
// The element chain is a linked list (each length says where the next element starts),
// which the reference walks one element at a time.  Here it is split into chunks of
// kNbChunk bytes.  The first element that starts in chunk c starts within GW_MAX_ELEMENT
// (= 64) bytes of the chunk start, so a wave per chunk walks all 64 candidate entries at
// once, one per lane (k_nb_walk).  Wrong candidates read payload bytes as lengths and
// die, or land on a real element start and merge with the true chain, so almost every
// chunk ends with one exit whatever its entry was.  k_nb_resolve then finds each chunk's
// true entry from the nearest chunk before it whose exit is unique, k_nb_scan turns the
// per-chunk record / watermark counts into output offsets, and k_nb_decode walks each
// chunk's true chain once more, out of LDS, and decodes its elements with all 64 lanes
// (byte-swaps, tag dispatch, coalesced column stores).
#include "gw_kernels.h"
#include "gw_netbuf.h"

namespace gw {

constexpr int kNbLanes = GW_MAX_ELEMENT;            // candidate entries per chunk (one per lane)
constexpr int kNbWaves = 4;                         // chunks per block
constexpr int kNbLds = kNbChunk + kNbLanes;         // chunk bytes + the overhang a length word may need
constexpr int kNbMaxElems = kNbChunk / 6 + 2;       // shortest element: 4 + RecordAttributes(2)

// lane state packed into the top byte of an exit word
constexpr int kStNormal = 0, kStTail = 1, kStDead = 2, kStLong = 3;
__device__ __forceinline__ int64_t nb_pack(int64_t pos, int st) { return pos | ((int64_t)st << 56); }
__host__ __device__ __forceinline__ int64_t nb_pos(int64_t w) { return w & (((int64_t)1 << 56) - 1); }
__host__ __device__ __forceinline__ int nb_state(int64_t w) { return (int)(w >> 56); }
constexpr int64_t kNonConv = -1;

// Stage bytes [base, base + kNbLds) ∩ [0, nbytes) of the buffer into LDS (one wave).
__device__ __forceinline__ void nb_stage(uint8_t* lds, const uint8_t* buf, int64_t base, int64_t nbytes) {
    const int lane = __lane_id();
    const int64_t avail = nbytes - base < kNbLds ? nbytes - base : kNbLds;
    const int words = (int)(avail >> 2);
    const uint32_t* src = (const uint32_t*)(buf + base);  // base is a multiple of kNbChunk; buf 4-aligned
    uint32_t* dst = (uint32_t*)lds;
    for (int i = lane; i < words; i += 64) dst[i] = __builtin_nontemporal_load(src + i);
    for (int i = words * 4 + lane; i < avail; i += 64) lds[i] = buf[base + i];
}

__device__ __forceinline__ uint32_t lds_be32(const uint8_t* l, int p) {
    return ((uint32_t)l[p] << 24) | ((uint32_t)l[p + 1] << 16) | ((uint32_t)l[p + 2] << 8) | (uint32_t)l[p + 3];
}
__device__ __forceinline__ uint64_t lds_be(const uint8_t* l, int p, int w) {
    uint64_t v = 0;
    for (int i = 0; i < w; ++i) v = (v << 8) | l[p + i];
    return v;
}

__global__ void __launch_bounds__(256) k_nb_walk(const uint8_t* buf, int64_t nbytes, int64_t nch, int64_t* exits,
                                                 int32_t* cnt, int64_t* conv) {
    __shared__ uint8_t lds[kNbWaves][kNbLds];
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const int64_t c = (int64_t)blockIdx.x * kNbWaves + w;
    if (c >= nch) return;  // whole wave
    const int64_t base = c * kNbChunk;
    nb_stage(lds[w], buf, base, nbytes);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t cend = base + kNbChunk < nbytes ? base + kNbChunk : nbytes;
    int64_t pos = base + lane;
    int nr = 0, nw = 0, st = kStNormal;
    while (pos < cend) {
        if (pos + 4 > nbytes) { st = kStTail; break; }
        const int32_t len = (int32_t)lds_be32(lds[w], (int)(pos - base));
        if (len < 1) { st = kStDead; break; }
        if (len > kNbLanes - 4) { st = kStLong; break; }
        if (pos + 4 + len > nbytes) { st = kStTail; break; }
        const int tag = lds[w][pos - base + 4];
        nr += tag <= 1;
        nw += tag == 2 || tag == 6;
        pos += 4 + len;
    }
    const int64_t ex = nb_pack(pos, st);
    exits[c * kNbLanes + lane] = ex;
    cnt[(c * kNbLanes + lane) * 2] = nr;
    cnt[(c * kNbLanes + lane) * 2 + 1] = nw;
    // unique exit over the live candidates (dead ones never hold the true entry)
    const bool live = st == kStNormal || st == kStTail;
    const unsigned long long lv = __ballot(live);
    int64_t cv = kNonConv;
    if (lv) {
        const int first = __ffsll((long long)lv) - 1;
        const int64_t ref = __shfl(ex, first);
        if (__ballot(live && ex != ref) == 0) cv = ref;
    } else {
        cv = nb_pack(base, kStDead);
    }
    if (lane == 0) conv[c] = cv;
}

// One thread per chunk: its true entry, from the nearest earlier chunk with a unique exit.
__global__ void __launch_bounds__(256) k_nb_resolve(int64_t nbytes, int64_t nch, const int64_t* exits,
                                                    const int32_t* cnt, const int64_t* conv, int64_t* entry,
                                                    int32_t* counts, NbStatus* st) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= nch) return;
    int64_t j = c - 1;
    while (j >= 0 && conv[j] == kNonConv) --j;
    int64_t e = j < 0 ? nb_pack(0, kStNormal) : conv[j];  // entry word of chunk j + 1
    for (int64_t t = j + 1; t < c && nb_state(e) == kStNormal; ++t) {
        const int64_t lane = nb_pos(e) - t * kNbChunk;
        if (lane < 0 || lane >= kNbLanes) { e = nb_pack(nb_pos(e), kStDead); break; }
        e = exits[t * kNbLanes + lane];
    }
    int32_t nr = 0, nw = 0;
    int64_t ent = -1;
    if (nb_state(e) == kStNormal) {
        const int64_t p = nb_pos(e);
        const int64_t lane = p - c * kNbChunk;
        if (p >= nbytes) {
            // the chain ended exactly at the end of the bytes: nothing starts here
        } else if (lane < 0 || lane >= kNbLanes) {
            atomicOr(&st->corrupt, 1ull);
        } else {
            ent = p;
            const int64_t ex = exits[c * kNbLanes + lane];
            nr = cnt[(c * kNbLanes + lane) * 2];
            nw = cnt[(c * kNbLanes + lane) * 2 + 1];
            const int s = nb_state(ex);
            if (s == kStDead) atomicOr(&st->corrupt, 1ull);
            if (s == kStLong) atomicOr(&st->unsupported, 1ull);
            if (s == kStTail) st->consumed = nb_pos(ex);  // at most one chunk of the chain stops early
            if (s == kStNormal && nb_pos(ex) >= nbytes) st->consumed = nbytes;
        }
    }
    entry[c] = ent;
    counts[2 * c] = nr;
    counts[2 * c + 1] = nw;
}

// Exclusive scan of the per-chunk (records, watermarks) counts; one block.
__global__ void __launch_bounds__(1024) k_nb_scan(int64_t nch, const int32_t* counts, int64_t* offs, NbStatus* st) {
    __shared__ long long part[1024][2];
    const int64_t per = (nch + blockDim.x - 1) / blockDim.x;
    const int64_t lo = threadIdx.x * per, hi = lo + per < nch ? lo + per : nch;
    long long r = 0, w = 0;
    for (int64_t i = lo; i < hi; ++i) { r += counts[2 * i]; w += counts[2 * i + 1]; }
    part[threadIdx.x][0] = r;
    part[threadIdx.x][1] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long a = 0, b = 0;
        for (int i = 0; i < (int)blockDim.x; ++i) {
            const long long x = part[i][0], y = part[i][1];
            part[i][0] = a; part[i][1] = b;
            a += x; b += y;
        }
        st->records = a;
        st->watermarks = b;
    }
    __syncthreads();
    r = part[threadIdx.x][0];
    w = part[threadIdx.x][1];
    for (int64_t i = lo; i < hi; ++i) {
        offs[2 * i] = r;
        offs[2 * i + 1] = w;
        r += counts[2 * i];
        w += counts[2 * i + 1];
    }
}

// field -> 8-byte column word (integral: sign-extended int64; float: widened double)
__device__ __forceinline__ int64_t nb_field(const uint8_t* l, int p, int type) {
    switch (type) {
    case 'J': case 'D': return (int64_t)lds_be(l, p, 8);
    case 'I': return (int64_t)(int32_t)(uint32_t)lds_be(l, p, 4);
    case 'S': return (int64_t)(int16_t)(uint16_t)lds_be(l, p, 2);
    case 'B': return (int64_t)(int8_t)l[p];
    case 'Z': return (int64_t)(l[p] != 0);
    case 'F': return f64_to_bits((double)__builtin_bit_cast(float, (uint32_t)lds_be(l, p, 4)));
    default: return 0;
    }
}

__global__ void __launch_bounds__(256) k_nb_decode(const uint8_t* buf, int64_t nbytes, int64_t nch, NbLayout L,
                                                   const int64_t* entry, const int64_t* offs, int64_t* key,
                                                   int64_t* ts, int64_t* val, int64_t rec_cap, int64_t* wm_pos,
                                                   int64_t* wm_val, int64_t wm_cap, NbStatus* st) {
    __shared__ uint8_t lds[kNbWaves][kNbLds];
    __shared__ uint16_t starts[kNbWaves][kNbMaxElems];
    __shared__ int nelem[kNbWaves];
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const int64_t c = (int64_t)blockIdx.x * kNbWaves + w;
    if (c >= nch) return;  // whole wave
    const int64_t e0 = entry[c];
    if (e0 < 0) return;
    const int64_t base = c * kNbChunk;
    nb_stage(lds[w], buf, base, nbytes);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint8_t* l = lds[w];
    const int64_t cend = base + kNbChunk < nbytes ? base + kNbChunk : nbytes;
    if (lane == 0) {  // the true chain (k_nb_walk proved every step of it is in bounds)
        int m = 0;
        int64_t pos = e0;
        for (; pos < cend && m < kNbMaxElems;) {
            if (pos + 4 > nbytes) break;
            const int32_t len = (int32_t)lds_be32(l, (int)(pos - base));
            if (len < 1 || len > kNbLanes - 4 || pos + 4 + len > nbytes) break;
            starts[w][m++] = (uint16_t)(pos - base);
            pos += 4 + len;
        }
        // more elements than valid ones of >= 6 bytes can make: lengths of 1 -> corrupt
        if (m == kNbMaxElems && pos < cend) atomicOr(&st->corrupt, 1ull);
        nelem[w] = m;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int m = nelem[w];
    int64_t rbase = offs[2 * c], wbase = offs[2 * c + 1];
    unsigned long long bad = 0, full = 0, skipped = 0;
    for (int i0 = 0; i0 < m; i0 += 64) {
        const int i = i0 + lane;
        int kind = 0;  // 0 none, 1 record, 2 watermark, 3 skipped
        int p = 0, len = 0, tag = -1;
        bool ok = true;  // the element's length matches its tag: its body lies inside the element
        if (i < m) {
            p = starts[w][i];
            len = (int)lds_be32(l, p);
            tag = l[p + 4];
            if (tag == 0 || tag == 1) {
                kind = 1;
                ok = len == (tag == 0 ? 9 : 1) + L.vbytes;
            } else if (tag == 2 || tag == 6) {
                kind = 2;
                ok = len == (tag == 2 ? 9 : 13);
            } else if (tag == 3 || tag == 4 || tag == 5) {
                kind = 3;
                ok = len == (tag == 3 ? 29 : tag == 4 ? 5 : 2);
            } else {
                ok = false;
            }
            if (!ok) bad = 1;
        }
        const unsigned long long below = (1ull << lane) - 1ull;
        const unsigned long long br = __ballot(kind == 1), bw = __ballot(kind == 2);
        skipped += kind == 3;
        if (kind == 1 && ok) {
            const int64_t o = rbase + __popcll(br & below);
            if (o < rec_cap) {
                const int hdr = tag == 0 ? 9 : 1;
                const int v = p + 4 + hdr;
                ts[o] = tag == 0 ? (int64_t)lds_be(l, p + 5, 8) : INT64_MIN;
                key[o] = (int64_t)lds_be(l, v + L.key_off, 8);
                if (val) val[o] = L.val_type ? nb_field(l, v + L.val_off, L.val_type) : 0;
            } else {
                full = 1;
            }
        } else if (kind == 2 && ok) {
            const int64_t o = wbase + __popcll(bw & below);
            if (o < wm_cap) {
                // records of this chunk before the watermark: those of lower lanes and earlier rounds
                wm_pos[o] = rbase + __popcll(br & below);
                wm_val[o] = (int64_t)lds_be(l, p + (tag == 2 ? 5 : 9), 8);
            } else {
                full = 1;
            }
        }
        rbase += __popcll(br);
        wbase += __popcll(bw);
    }
    bad = wave_ior(bad);
    full = wave_ior(full);
    skipped = wave_sum(skipped);
    if (lane == 0) {
        if (bad) atomicOr(&st->corrupt, 1ull);
        if (full) atomicOr(&st->full, 1ull);
        if (skipped) atomicAdd(&st->skipped, skipped);
    }
}

int64_t nb_scratch_bytes(int64_t nbytes) {
    const int64_t nch = (nbytes + kNbChunk - 1) / kNbChunk;
    // exits, per-lane counts, conv, entry, per-chunk counts, offsets, status
    return nch * kNbLanes * 8 + nch * kNbLanes * 8 + nch * 8 + nch * 8 + nch * 8 + nch * 16 + 256;
}

hipError_t launch_nb_decode(const uint8_t* buf, int64_t nbytes, const NbLayout& L, int64_t* key, int64_t* ts,
                            int64_t* val, int64_t rec_cap, int64_t* wm_pos, int64_t* wm_val, int64_t wm_cap,
                            void* scratch, NbStatus* d_st, hipStream_t s) {
    hipError_t e = hipMemsetAsync(d_st, 0, sizeof(NbStatus), s);
    if (e != hipSuccess || nbytes <= 0) return e;
    const int64_t nch = (nbytes + kNbChunk - 1) / kNbChunk;
    uint8_t* p = (uint8_t*)scratch;
    int64_t* exits = (int64_t*)p;              p += nch * kNbLanes * 8;
    int32_t* cnt = (int32_t*)p;                p += nch * kNbLanes * 8;
    int64_t* conv = (int64_t*)p;               p += nch * 8;
    int64_t* entry = (int64_t*)p;              p += nch * 8;
    int32_t* counts = (int32_t*)p;             p += nch * 8;
    int64_t* offs = (int64_t*)p;
    const unsigned gb = (unsigned)((nch + kNbWaves - 1) / kNbWaves);
    hipLaunchKernelGGL(k_nb_walk, dim3(gb), dim3(256), 0, s, buf, nbytes, nch, exits, cnt, conv);
    hipLaunchKernelGGL(k_nb_resolve, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, nbytes, nch, exits, cnt,
                       conv, entry, counts, d_st);
    hipLaunchKernelGGL(k_nb_scan, dim3(1), dim3(1024), 0, s, nch, counts, offs, d_st);
    hipLaunchKernelGGL(k_nb_decode, dim3(gb), dim3(256), 0, s, buf, nbytes, nch, L, entry, offs, key, ts, val, rec_cap,
                       wm_pos, wm_val, wm_cap, d_st);
    return hipGetLastError();
}

}  // namespace gw
