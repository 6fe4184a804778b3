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
// kNbChunk bytes.  The first element that starts in chunk c starts within the longest
// element (NL = 64 bytes, or 128 = GW_MAX_ELEMENT for layouts whose records are longer)
// of the chunk start, so a wave per chunk walks all NL candidate entries at once, one or
// two per lane (k_nb_walk).  Wrong candidates read payload bytes as lengths and
// die, or land on a real element start and merge with the true chain, so almost every
// chunk ends with one exit whatever its entry was.  k_nb_resolve then finds each chunk's
// true entry from the nearest chunk before it whose exit is unique, k_nb_scan turns the
// per-chunk record / watermark counts into output offsets, and k_nb_decode walks each
// chunk's true chain once more, out of LDS, and decodes its elements with all 64 lanes
// (byte-swaps, tag dispatch, coalesced column stores).
#include <cstdlib>

#include "gw_kernels.h"
#include "gw_netbuf.h"

namespace gw {

// NL: candidate entries per chunk = the longest element (64, or GW_MAX_ELEMENT = 128 when
// the record layout's elements exceed 64 bytes); NL / 64 candidates per lane.
constexpr int kNbWaves = 4;                              // chunks per block
template <int NL>
constexpr int nb_words() { return (kNbChunk + NL + 8) / 4; }  // chunk + overhang + one spare dword
constexpr int kNbMaxElems = kNbChunk / 6 + 2;            // shortest element: 4 + RecordAttributes(2)
constexpr int kNbScanBlock = 256;                        // chunks per k_nb_resolve block
constexpr int kNbMaxLanes = GW_MAX_ELEMENT;              // scratch sizing: the widest walk
constexpr int kNbMaskWords = kNbChunk / 32;              // element-start mask words per chunk
// sync window: bytes of a chunk the candidates walk before checking that they agree
#ifndef GW_NB_SYNC
#define GW_NB_SYNC 80  // walk per 10M Q5 records: 256 B 204 us, 128 B 125 us, 96 B 98 us (8 fallback chunks),
                       // 80 B 91 us (55), 72 B 89 us (191)
#endif
template <int NL>
constexpr int nb_sync_bytes() { return NL == 64 ? GW_NB_SYNC : 2 * GW_NB_SYNC; }

// walk state of a candidate lane, packed into the top bits of its exit word
constexpr int kStNormal = 0, kStTail = 1, kStDead = 2, kStLong = 3;
__device__ __forceinline__ int64_t nb_pack(int64_t pos, int st) { return pos | ((int64_t)st << 56); }
__device__ __forceinline__ int64_t nb_pos(int64_t w) { return w & (((int64_t)1 << 56) - 1); }
__device__ __forceinline__ int nb_state(int64_t w) { return (int)(w >> 56); }
constexpr int64_t kNonConv = -1;

// A wave's chunk in flight: bytes [base, base + 4*kNbWords) ∩ [0, nbytes) as dwords in
// registers (kNbRegs per lane; bytes past the end read as 0), loaded one chunk ahead of
// the walk so the HBM latency hides behind the LDS chain walk of the current chunk.
template <int NL>
constexpr int nb_regs() { return (nb_words<NL>() + 63) / 64; }
template <int NL>
__device__ __forceinline__ void nb_fetch(uint32_t (&r)[nb_regs<NL>()], const uint8_t* buf, int64_t base,
                                         int64_t nbytes) {
    constexpr int kNbWords = nb_words<NL>(), kNbRegs = nb_regs<NL>();
    const int lane = __lane_id();
    const int64_t left = nbytes - base;
    const uint32_t* src = (const uint32_t*)(buf + base);  // base is a multiple of kNbChunk; buf 4-aligned
    if (left >= 4 * (int64_t)(64 * kNbRegs)) {  // the whole register window is in range (wave-uniform)
#pragma unroll
        for (int k = 0; k < kNbRegs; ++k) r[k] = __builtin_nontemporal_load(src + lane + 64 * k);
        return;
    }
    const int avail = left < 4 * kNbWords ? (int)left : 4 * kNbWords;
    const int full = avail >> 2;
#pragma unroll
    for (int k = 0; k < kNbRegs; ++k) {
        const int i = lane + 64 * k;
        uint32_t v = 0;
        if (i < full) {
            v = __builtin_nontemporal_load(src + i);
        } else if (i == full) {
            for (int b = 0; b < (avail & 3); ++b) v |= (uint32_t)buf[base + 4 * i + b] << (8 * b);
        }
        r[k] = v;
    }
}
template <int NL>
__device__ __forceinline__ void nb_put(uint32_t* lds, const uint32_t (&r)[nb_regs<NL>()]) {
    constexpr int kNbWords = nb_words<NL>(), kNbRegs = nb_regs<NL>();
    const int lane = __lane_id();
#pragma unroll
    for (int k = 0; k < kNbRegs; ++k) {
        const int i = lane + 64 * k;
        if (i < kNbWords) lds[i] = r[k];
    }
}

// Little-endian dwords in LDS -> big-endian fields at any byte offset p.
__device__ __forceinline__ uint32_t lds_le32(const uint32_t* w, int p) {
    const int q = p >> 2;
    return __builtin_amdgcn_alignbyte(w[q + 1], w[q], (uint32_t)(p & 3));
}
__device__ __forceinline__ uint32_t lds_be32(const uint32_t* w, int p) { return __builtin_bswap32(lds_le32(w, p)); }
__device__ __forceinline__ uint32_t lds_byte(const uint32_t* w, int p) { return (w[p >> 2] >> (8 * (p & 3))) & 0xffu; }
__device__ __forceinline__ uint64_t lds_be64(const uint32_t* w, int p) {
    const int q = p >> 2;
    const uint32_t r = (uint32_t)(p & 3);
    const uint32_t w0 = w[q], w1 = w[q + 1], w2 = w[q + 2];
    const uint64_t le = ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, r) << 32) | __builtin_amdgcn_alignbyte(w1, w0, r);
    return __builtin_bswap64(le);
}

// One candidate's walk from its state (pos, counts, st) while pos < H, out of LDS.
// Branch-free step (one ds_read2 gives the length word and the tag): every lane steps in
// lockstep under a full exec mask, and the per-step VALU count stays small.
__device__ __forceinline__ void nb_walk_lane(const uint32_t* l, int H, int rlim, int rec_ts, int rec_nots, bool run,
                                             int& pos, uint32_t& cnt, int& st) {
    while (__ballot(run)) {
        const int p = run ? pos : 0;
        const uint32_t w0 = l[p >> 2], w1 = l[(p >> 2) + 1];
        const uint32_t sh = (uint32_t)(p & 3);
        const int32_t len = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, sh));
        const uint32_t tag = (w1 >> (8 * sh)) & 0xffu;
        // a candidate lives only on elements whose length fits their tag (what k_nb_decode
        // checks on the true chain): payload bytes that merely read as a plausible length
        // rarely also carry the matching tag, so wrong chains die within a step or two
        // the length each tag's element must have, as bytes of two words (tag 7: 255, which
        // no element reaches: GW_MAX_ELEMENT)
        const uint32_t lut = (tag & 4u) ? (5u | 2u << 8 | 13u << 16 | 255u << 24)
                                        : ((uint32_t)rec_ts | (uint32_t)rec_nots << 8 | 9u << 16 | 29u << 24);
        const int want = tag < 8u ? (int)((lut >> (8 * (tag & 3u))) & 0xffu) : -1;
        // beyond GW_MAX_ELEMENT: unsupported; longer than NL but within it: no element of
        // this layout is that long, so the length cannot match its tag (dead: corrupt on
        // the true chain) -- the same order of checks as the oracle's decoder
        const int ns = p + 4 > rlim ? kStTail
                     : len < 1 ? kStDead
                     : len > GW_MAX_ELEMENT - 4 ? kStLong
                     : p + 4 + len > rlim ? kStTail
                     : len != want ? kStDead : kStNormal;
        const bool adv = run && ns == kStNormal;
        st = (run && !adv) ? ns : st;
        // records | watermarks << 16 in one word: 2-bit class per tag (0, 1: record; 2, 6:
        // watermark; 3-5: skipped), from a packed table
        const uint32_t cls = (0x2025u >> (2 * (tag & 7u))) & 3u;
        cnt += adv ? ((cls & 1u) | ((cls & 2u) << 15)) : 0u;
        pos = adv ? p + 4 + len : pos;
        run = adv && pos < H;
    }
}

// Pass 1: every candidate entry of every chunk (lane = candidate offset, plus 64 for the
// second candidate of a lane when NL = 128), walked at once -- but only through a short
// sync window of the chunk's first kNbSync bytes.  Wrong candidates die or merge within
// a step or two, so at the window's end the live candidates almost always stand on one
// element start P of the true chain (whatever the entry): then the chunk records P
// (sync), each candidate's (P or its death, counts up to P), and k_nb_tail walks P to the
// chunk's end with one thread.  Otherwise (a payload that mimics a chain for longer, the
// stream's last chunk) the wave loads the whole chunk and walks on to its end, as before.
// Per candidate: exit (relative position | state << 28) and (records | watermarks << 16).
template <int NL>
__global__ void __launch_bounds__(256) k_nb_walk(const uint8_t* buf, int64_t nbytes, int64_t nch, int32_t vbytes,
                                                 uint32_t* exits, uint32_t* cnt, int64_t* conv, int64_t* sync,
                                                 NbStatus* nst) {
    constexpr int kNbWords = nb_words<NL>(), CPL = NL / 64;
    constexpr int kSyncWords = nb_sync_bytes<NL>() / 4, kSyncRegs = (kSyncWords + 63) / 64;
    constexpr int kSync = nb_sync_bytes<NL>() - 8;
    const int rec_ts = 9 + vbytes, rec_nots = 1 + vbytes;
    __shared__ uint32_t lds[kNbWaves][kNbWords];
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const int64_t stride = (int64_t)gridDim.x * kNbWaves;
    uint32_t pre[kSyncRegs];
    auto fetch_window = [&](int64_t b) {  // the sync window's dwords (bytes past the end read as 0)
        const int64_t left = nbytes - b;
        const uint32_t* src = (const uint32_t*)(buf + b);
        if (left >= 4 * (int64_t)(64 * kSyncRegs)) {  // in range (wave-uniform)
#pragma unroll
            for (int k = 0; k < kSyncRegs; ++k)
                pre[k] = lane + 64 * k < kSyncWords ? __builtin_nontemporal_load(src + lane + 64 * k) : 0u;
            return;
        }
#pragma unroll
        for (int k = 0; k < kSyncRegs; ++k) {
            const int i = lane + 64 * k;
            uint32_t v = 0;
            if (i >= kSyncWords) {
            } else if (4 * (int64_t)i + 4 <= left) {
                v = __builtin_nontemporal_load(src + i);
            } else {
                for (int q = 0; q < 4; ++q)
                    if (4 * (int64_t)i + q < left) v |= (uint32_t)buf[b + 4 * i + q] << (8 * q);
            }
            pre[k] = v;
        }
    };
    int64_t c = (int64_t)blockIdx.x * kNbWaves + w;
    if (c < nch) fetch_window(c * kNbChunk);
    for (; c < nch; c += stride) {
    const int64_t base = c * kNbChunk;
    __builtin_amdgcn_wave_barrier();  // the previous chunk's LDS reads are done
#pragma unroll
    for (int k = 0; k < kSyncRegs; ++k)
        if (lane + 64 * k < kSyncWords) lds[w][lane + 64 * k] = pre[k];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (c + stride < nch) fetch_window((c + stride) * kNbChunk);
    const uint32_t* l = lds[w];
    const int64_t left = nbytes - base;
    const int rlim = left < kNbChunk + 4 * NL ? (int)left : kNbChunk + 4 * NL;  // binding only near the end
    const int rend = rlim < kNbChunk ? rlim : kNbChunk;
    const bool windowed = rend > kSync;
    const int H = windowed ? kSync : rend;
    int pos[CPL], st[CPL];
    uint32_t cn[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        pos[k] = lane + 64 * k; cn[k] = 0; st[k] = kStNormal;
        nb_walk_lane(l, H, rlim, rec_ts, rec_nots, pos[k] < H, pos[k], cn[k], st[k]);
    }
    // converged: every live candidate stopped normally on the same position
    bool conv_ok = windowed;
    int P = -1;
    if (windowed) {
        unsigned long long anyl = 0;
#pragma unroll
        for (int k = 0; k < CPL; ++k) anyl |= __ballot(st[k] == kStNormal || st[k] == kStTail);
        if (!anyl) {
            conv_ok = false;  // no live candidate: dead everywhere (the full walk changes nothing)
        } else {
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const unsigned long long lv = __ballot(st[k] == kStNormal);
                if (P < 0 && lv) P = __shfl(pos[k], __ffsll((long long)lv) - 1);
            }
            bool diff = false;
#pragma unroll
            for (int k = 0; k < CPL; ++k)
                diff = diff || __ballot(st[k] == kStTail || (st[k] == kStNormal && pos[k] != P)) != 0;
            conv_ok = !diff && P >= 0;
        }
    }
    if (windowed && !conv_ok) {  // walk on to the chunk's end out of the whole chunk
        if (lane == 0) atomicAdd(&nst->fallback, 1ull);
        uint32_t full[nb_regs<NL>()];
        nb_fetch<NL>(full, buf, base, nbytes);
        __builtin_amdgcn_wave_barrier();
        nb_put<NL>(lds[w], full);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            nb_walk_lane(l, rend, rlim, rec_ts, rec_nots, st[k] == kStNormal && pos[k] < rend, pos[k], cn[k], st[k]);
    }
    int64_t ex[CPL];
    bool live[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int cand = lane + 64 * k;
        exits[c * NL + cand] = (uint32_t)pos[k] | ((uint32_t)st[k] << 28);
        cnt[c * NL + cand] = cn[k];
        ex[k] = nb_pack(base + pos[k], st[k]);
        live[k] = st[k] == kStNormal || st[k] == kStTail;
    }
    if (conv_ok) {  // k_nb_tail finishes the chain from P and writes conv[c]
        if (lane == 0) sync[c] = base + P;
        continue;
    }
    // unique exit over the live candidates (dead ones never hold the true entry)
    int64_t ref = 0;
    bool have = false;
#pragma unroll
    for (int k = 0; k < CPL && !have; ++k) {
        const unsigned long long lv = __ballot(live[k]);
        if (lv) {
            ref = __shfl(ex[k], __ffsll((long long)lv) - 1);
            have = true;
        }
    }
    int64_t cv = nb_pack(base, kStDead);
    if (have) {
        bool diff = false;
#pragma unroll
        for (int k = 0; k < CPL; ++k) diff = diff || __ballot(live[k] && ex[k] != ref) != 0;
        cv = diff ? kNonConv : ref;
    }
    if (lane == 0) {
        conv[c] = cv;
        sync[c] = -1;
    }
    }
}

// Pass 1b: one thread per synced chunk walks the true chain from its sync point P to the
// chunk's end (global loads; each thread streams through its own chunk), the exit and the
// record / watermark counts of [P, exit) -> conv[c], tcnt[c], the element starts -> tmask.
template <int NL>
__global__ void __launch_bounds__(256) k_nb_tail(const uint8_t* buf, int64_t nbytes, int64_t nch, int32_t vbytes,
                                                 const int64_t* sync, int64_t* conv, uint32_t* tcnt,
                                                 uint32_t* tmask) {
    // element starts of [P, exit) as a bit mask per chunk (kNbMaskWords words), which
    // k_nb_decode expands with all lanes instead of walking the chain again; staged in LDS
    // (one row per thread, padded against bank conflicts) and written out coalesced
    constexpr int kRow = kNbMaskWords + 1;
    __shared__ uint32_t lm[256 * kRow];
    const int rec_ts = 9 + vbytes, rec_nots = 1 + vbytes;
    const int tid = threadIdx.x;
    for (int64_t c0 = (int64_t)blockIdx.x * 256; c0 < nch; c0 += (int64_t)gridDim.x * 256) {
        const int64_t c = c0 + tid;
        uint32_t* mk = lm + tid * kRow;
        const int64_t s0 = c < nch ? sync[c] : -1;
        if (s0 >= 0) {
            const int64_t base = c * kNbChunk;
            const int64_t left = nbytes - base;
            const int rlim = left < kNbChunk + 4 * NL ? (int)left : kNbChunk + 4 * NL;
            const int rend = rlim < kNbChunk ? rlim : kNbChunk;
            const uint8_t* b = buf + base;
            int pos = (int)(s0 - base), nr = 0, nw = 0, st = kStNormal, mw = 0;
            uint32_t cur = 0;
            while (pos < rend) {
                if (pos + 4 > rlim) { st = kStTail; break; }
                int32_t len;
                uint32_t tag;
                const int q = pos & ~3;
                if ((int64_t)q + 8 <= left) {  // one 8-byte load holds the length word and the tag
                    const uint2 d = *(const uint2*)(b + q);
                    const uint32_t sh = (uint32_t)(pos & 3);
                    len = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(d.y, d.x, sh));
                    tag = (d.y >> (8 * sh)) & 0xffu;
                } else {
                    len = (int32_t)(((uint32_t)b[pos] << 24) | ((uint32_t)b[pos + 1] << 16) |
                                    ((uint32_t)b[pos + 2] << 8) | (uint32_t)b[pos + 3]);
                    tag = pos + 4 < left ? b[pos + 4] : 0u;
                }
                const int want = tag == 0u ? rec_ts : tag == 1u ? rec_nots : tag == 2u ? 9 : tag == 3u ? 29
                               : tag == 4u ? 5 : tag == 5u ? 2 : tag == 6u ? 13 : -1;
                const int ns = len < 1 ? kStDead
                             : len > GW_MAX_ELEMENT - 4 ? kStLong
                             : pos + 4 + len > rlim ? kStTail
                             : len != want ? kStDead : kStNormal;
                if (ns != kStNormal) { st = ns; break; }
                nr += tag <= 1u ? 1 : 0;
                nw += (tag == 2u || tag == 6u) ? 1 : 0;
                for (; mw < (pos >> 5); ++mw, cur = 0) mk[mw] = cur;
                cur |= 1u << (pos & 31);
                pos += 4 + len;
            }
            for (; mw < kNbMaskWords; ++mw, cur = 0) mk[mw] = cur;
            conv[c] = nb_pack(base + pos, st);
            tcnt[c] = (uint32_t)nr | ((uint32_t)nw << 16);
        } else {
            for (int k = 0; k < kNbMaskWords; ++k) mk[k] = 0;
        }
        __syncthreads();
        const int64_t nrow = nch - c0 < 256 ? nch - c0 : 256;
        for (int j = tid; j < nrow * kNbMaskWords; j += 256)
            tmask[c0 * kNbMaskWords + j] = lm[(j / kNbMaskWords) * kRow + j % kNbMaskWords];
        __syncthreads();
    }
}

// A candidate's exit from chunk t: its walk's end, or for a synced chunk whose candidate
// reached the sync point, the tail walk's end.
template <int NL>
__device__ __forceinline__ int64_t nb_exit_word(const uint32_t* exits, const int64_t* sync, const int64_t* conv,
                                                int64_t t, int64_t lane) {
    const uint32_t x = exits[t * NL + lane];
    const int64_t e = nb_pack(t * kNbChunk + (x & 0x0fffffffu), (int)(x >> 28));
    return (sync[t] >= 0 && e == nb_pack(sync[t], kStNormal)) ? conv[t] : e;
}

// Pass 2: one thread per chunk finds its true entry from the nearest earlier chunk with a
// unique exit, then the block scans the chunk counts (exclusive, block-local).
template <int NL>
__global__ void __launch_bounds__(kNbScanBlock) k_nb_resolve(int64_t nbytes, int64_t nch, const uint32_t* exits,
                                                             const uint32_t* cnt, const int64_t* conv,
                                                             const int64_t* sync, const uint32_t* tcnt, int64_t* entry,
                                                             int32_t* offs, long long* btot, NbStatus* st) {
    __shared__ int wsum[kNbScanBlock / 64][2];
    const int64_t c = (int64_t)blockIdx.x * kNbScanBlock + threadIdx.x;
    int nr = 0, nw = 0;
    if (c < nch) {
        int64_t j = c - 1;
        while (j >= 0 && conv[j] == kNonConv) --j;
        if (j < c - 1) atomicAdd(&st->walkback, (unsigned long long)(c - 1 - j));
        int64_t e = j < 0 ? nb_pack(0, kStNormal) : conv[j];  // entry word of chunk j + 1
        for (int64_t t = j + 1; t < c && nb_state(e) == kStNormal; ++t) {
            const int64_t lane = nb_pos(e) - t * kNbChunk;
            if (lane < 0 || lane >= NL) { e = nb_pack(nb_pos(e), kStDead); break; }
            e = nb_exit_word<NL>(exits, sync, conv, t, lane);
        }
        int64_t ent = -1;
        if (nb_state(e) == kStNormal) {
            const int64_t p = nb_pos(e);
            const int64_t lane = p - c * kNbChunk;
            if (p >= nbytes) {
                // the chain ended exactly at the end of the bytes: nothing starts here
            } else if (lane < 0 || lane >= NL) {
                atomicOr(&st->corrupt, 1ull);
            } else {
                ent = p;
                const int64_t ex = nb_exit_word<NL>(exits, sync, conv, c, lane);
                const uint32_t cc = cnt[c * NL + lane];
                nr = (int)(cc & 0xffffu);
                nw = (int)(cc >> 16);
                const uint32_t x = exits[c * NL + lane];
                if (sync[c] >= 0 && nb_pack(c * kNbChunk + (x & 0x0fffffffu), (int)(x >> 28)) ==
                                        nb_pack(sync[c], kStNormal)) {
                    nr += (int)(tcnt[c] & 0xffffu);
                    nw += (int)(tcnt[c] >> 16);
                }
                const int s = nb_state(ex);
                if (s == kStDead) atomicOr(&st->corrupt, 1ull);
                if (s == kStLong) atomicOr(&st->unsupported, 1ull);
                if (s == kStTail) st->consumed = nb_pos(ex);  // at most one chunk of the chain stops early
                if (s == kStNormal && nb_pos(ex) >= nbytes) st->consumed = nbytes;
            }
        }
        entry[c] = ent;
    }
    // block-local exclusive scan of (nr, nw): wave prefix, then across the 4 waves
    const int lane = __lane_id(), wv = threadIdx.x >> 6;
    int ir = nr, iw = nw;
    for (int o = 1; o < 64; o <<= 1) {
        const int ur = __shfl_up(ir, o), uw = __shfl_up(iw, o);
        if (lane >= o) { ir += ur; iw += uw; }
    }
    if (lane == 63) { wsum[wv][0] = ir; wsum[wv][1] = iw; }
    __syncthreads();
    int br = 0, bw = 0;
    for (int k = 0; k < wv; ++k) { br += wsum[k][0]; bw += wsum[k][1]; }
    if (c < nch) {
        offs[2 * c] = br + ir - nr;
        offs[2 * c + 1] = bw + iw - nw;
    }
    if (threadIdx.x == kNbScanBlock - 1) {
        btot[2 * blockIdx.x] = br + ir;
        btot[2 * blockIdx.x + 1] = bw + iw;
    }
}

// Pass 3: exclusive scan of the per-block totals (in place); one block.
__global__ void __launch_bounds__(1024) k_nb_scan(int64_t nblk, long long* btot, NbStatus* st) {
    __shared__ long long part[1024][2];
    const int64_t per = (nblk + blockDim.x - 1) / blockDim.x;
    const int64_t lo = threadIdx.x * per, hi = lo + per < nblk ? lo + per : nblk;
    long long r = 0, w = 0;
    for (int64_t i = lo; i < hi; ++i) { r += btot[2 * i]; w += btot[2 * i + 1]; }
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
        const long long x = btot[2 * i], y = btot[2 * i + 1];
        btot[2 * i] = r;
        btot[2 * i + 1] = w;
        r += x;
        w += y;
    }
}

// field -> 8-byte column word (integral: sign-extended int64; float: widened double)
__device__ __forceinline__ int64_t nb_field(const uint32_t* l, int p, int type) {
    switch (type) {
    case 'J': case 'D': return (int64_t)lds_be64(l, p);
    case 'I': return (int64_t)(int32_t)lds_be32(l, p);
    case 'S': return (int64_t)(int16_t)(uint16_t)(lds_be32(l, p) >> 16);
    case 'B': return (int64_t)(int8_t)(uint8_t)lds_byte(l, p);
    case 'Z': return (int64_t)(lds_byte(l, p) != 0);
    case 'F': return f64_to_bits((double)__builtin_bit_cast(float, lds_be32(l, p)));
    default: return 0;
    }
}

// Pass 4: each chunk's true chain, walked once more out of LDS, decoded by all 64 lanes.
template <int NL>
__global__ void __launch_bounds__(256) k_nb_decode(const uint8_t* buf, int64_t nbytes, int64_t nch, NbLayout L,
                                                   const int64_t* entry, const int32_t* offs, const long long* btot,
                                                   const int64_t* sync, const uint32_t* tmask,
                                                   int64_t* key, int64_t* ts, int64_t* val, int64_t rec_cap,
                                                   int64_t* wm_pos, int64_t* wm_val, int64_t wm_cap, NbStatus* st) {
    constexpr int kNbWords = nb_words<NL>(), kNbRegs = nb_regs<NL>();
    __shared__ uint32_t lds[kNbWaves][kNbWords];
    __shared__ uint16_t starts[kNbWaves][kNbMaxElems];
    __shared__ int nelem[kNbWaves];
    const int w = threadIdx.x >> 6, lane = __lane_id();
    const int64_t stride = (int64_t)gridDim.x * kNbWaves;
    uint32_t pre[kNbRegs];
    // the next chunk's entry, sync point, mask word and output offsets load with its bytes
    int64_t pe0 = -1, psy = -1, prb = 0, pwb = 0;
    uint32_t pmw = 0;
    auto fetch_meta = [&](int64_t cc) {
        pe0 = entry[cc];
        psy = sync[cc];
        pmw = lane < kNbMaskWords ? tmask[cc * kNbMaskWords + lane] : 0u;
        const int64_t blk = cc / kNbScanBlock;
        prb = btot[2 * blk] + offs[2 * cc];
        pwb = btot[2 * blk + 1] + offs[2 * cc + 1];
    };
    int64_t c = (int64_t)blockIdx.x * kNbWaves + w;
    if (c < nch) {
        nb_fetch<NL>(pre, buf, c * kNbChunk, nbytes);
        fetch_meta(c);
    }
    for (; c < nch; c += stride) {
    const int64_t e0 = pe0, sy = psy;
    const uint32_t mword = pmw;
    int64_t rbase = prb, wbase = pwb;
    const int64_t base = c * kNbChunk;
    __builtin_amdgcn_wave_barrier();  // the previous chunk's LDS reads are done
    nb_put<NL>(lds[w], pre);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (c + stride < nch) {
        nb_fetch<NL>(pre, buf, (c + stride) * kNbChunk, nbytes);
        fetch_meta(c + stride);
    }
    if (e0 < 0) continue;
    const uint32_t* l = lds[w];
    const int64_t left = nbytes - base;
    const int rlim = left < kNbChunk + 4 * NL ? (int)left : kNbChunk + 4 * NL;
    const int rend = rlim < kNbChunk ? rlim : kNbChunk;
    {  // the true chain, walked by the whole wave in lockstep (uniform addresses: LDS
       // broadcasts), lane 0 recording the element starts -- for a synced chunk only up to
       // its sync point P: the starts from P on come from k_nb_tail's mask
        int m = 0;
        int pos = (int)(e0 - base);
        const int P = sy >= 0 ? (int)(sy - base) : -1;
        bool run = pos < rend;
        while (run && m < kNbMaxElems && pos != P) {
            const uint32_t w0 = l[pos >> 2], w1 = l[(pos >> 2) + 1];
            const int32_t len = (int32_t)__builtin_bswap32(__builtin_amdgcn_alignbyte(w1, w0, (uint32_t)(pos & 3)));
            if (pos + 4 > rlim || len < 1 || len > NL - 4 || pos + 4 + len > rlim) break;
            if (lane == 0) starts[w][m] = (uint16_t)pos;
            ++m;
            pos += 4 + len;
            run = pos < rend;
        }
        if (run && pos == P) {  // expand the mask: lane k < kNbMaskWords holds word k
            uint32_t word = mword;
            const int nb = __popc(word);
            int incl = nb;
            for (int o = 1; o < 64; o <<= 1) {
                const int u = __shfl_up(incl, o);
                if (lane >= o) incl += u;
            }
            int at = m + incl - nb;
            while (word) {
                const int bit = __ffs(word) - 1;
                word &= word - 1;
                if (at < kNbMaxElems) starts[w][at] = (uint16_t)(lane * 32 + bit);
                ++at;
            }
            m += __shfl(incl, 63);
            pos = rend;  // (the tail's own end state was resolved by k_nb_resolve)
            if (m > kNbMaxElems) m = kNbMaxElems;
        }
        // more elements than valid ones of >= 6 bytes can make: lengths of 1 -> corrupt
        if (lane == 0 && m == kNbMaxElems && pos < rend) atomicOr(&st->corrupt, 1ull);
        if (lane == 0) nelem[w] = m;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int m = nelem[w];
    unsigned long long bad = 0, full = 0, skipped = 0;
    for (int i0 = 0; i0 < m; i0 += 64) {
        const int i = i0 + lane;
        int kind = 0;  // 0 none, 1 record, 2 watermark, 3 skipped
        int p = 0, len = 0, tag = -1;
        bool ok = true;  // the element's length matches its tag: its body lies inside the element
        if (i < m) {
            p = starts[w][i];
            len = (int)lds_be32(l, p);
            tag = (int)lds_byte(l, p + 4);
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
        skipped += (unsigned long long)__popcll(__ballot(kind == 3));  // wave-uniform
        if (kind == 1 && ok) {
            const int64_t o = rbase + __popcll(br & below);
            if (o < rec_cap) {
                const int hdr = tag == 0 ? 9 : 1;
                const int v = p + 4 + hdr;
                ts[o] = tag == 0 ? (int64_t)lds_be64(l, p + 5) : INT64_MIN;
                key[o] = (int64_t)lds_be64(l, v + L.key_off);
                if (val) val[o] = L.val_type ? nb_field(l, v + L.val_off, L.val_type) : 0;
            } else {
                full = 1;
            }
        } else if (kind == 2 && ok) {
            const int64_t o = wbase + __popcll(bw & below);
            if (o < wm_cap) {
                // records before the watermark: all earlier chunks', earlier rounds', lower lanes'
                wm_pos[o] = rbase + __popcll(br & below);
                wm_val[o] = (int64_t)lds_be64(l, p + (tag == 2 ? 5 : 9));
            } else {
                full = 1;
            }
        }
        rbase += __popcll(br);
        wbase += __popcll(bw);
    }
    bad = __ballot(bad != 0) != 0;  // one ballot each instead of a wave reduction
    full = __ballot(full != 0) != 0;
    if (lane == 0) {
        if (bad) atomicOr(&st->corrupt, 1ull);
        if (full) atomicOr(&st->full, 1ull);
        if (skipped) atomicAdd(&st->skipped, skipped);
    }
    }
}

int64_t nb_scratch_bytes(int64_t nbytes) {
    const int64_t nch = (nbytes + kNbChunk - 1) / kNbChunk;
    const int64_t nblk = (nch + kNbScanBlock - 1) / kNbScanBlock;
    // exits + counts per lane, conv + entry + offsets per chunk, block totals
    return nch * kNbMaxLanes * 8 + nch * (40 + 4 * kNbMaskWords) + nblk * 16 + 256;
}

hipError_t launch_nb_decode(const uint8_t* buf, int64_t nbytes, const NbLayout& L, int64_t* key, int64_t* ts,
                            int64_t* val, int64_t rec_cap, int64_t* wm_pos, int64_t* wm_val, int64_t wm_cap,
                            void* scratch, NbStatus* d_st, hipStream_t s) {
    hipError_t e = hipMemsetAsync(d_st, 0, sizeof(NbStatus), s);
    if (e != hipSuccess || nbytes <= 0) return e;
    const int64_t nch = (nbytes + kNbChunk - 1) / kNbChunk;
    const int64_t nblk = (nch + kNbScanBlock - 1) / kNbScanBlock;
    uint8_t* p = (uint8_t*)scratch;
    uint32_t* exits = (uint32_t*)p;            p += nch * kNbMaxLanes * 4;
    uint32_t* cnt = (uint32_t*)p;              p += nch * kNbMaxLanes * 4;
    int64_t* conv = (int64_t*)p;               p += nch * 8;
    int64_t* entry = (int64_t*)p;              p += nch * 8;
    int32_t* offs = (int32_t*)p;               p += nch * 8;
    int64_t* sync = (int64_t*)p;               p += nch * 8;
    uint32_t* tcnt = (uint32_t*)p;             p += nch * 8;
    uint32_t* tmask = (uint32_t*)p;            p += nch * 4 * kNbMaskWords;
    long long* btot = (long long*)p;
    // a bounded grid of waves that loop over the chunks: a chunk is ~1 us of work, too
    // little to pay for a workgroup dispatch each (GW_NB_GRID overrides, for sweeps)
    int64_t gb = (nch + kNbWaves - 1) / kNbWaves;
    static const int64_t cap = [] {
        const char* e = getenv("GW_NB_GRID");
        return e ? (int64_t)atoll(e) : (int64_t)8192;  // measured: 1024 / 2048 / 4096 / 8192 / uncapped
    }();                                                // decode 272 / 257 / 244 / 231 / 251 us
    if (cap > 0 && gb > cap) gb = cap;
    // tail walks: a grid of 512 blocks looping over the chunks (measured: 128 blocks 160 us,
    // 256 98 us, 512 86 us, 1024 86 us per 10M Q5 records)
    static const int64_t tcap = [] {
        const char* e = getenv("GW_NB_TAIL_GRID");
        return e ? (int64_t)atoll(e) : (int64_t)512;
    }();
    int64_t tb = (nch + 255) / 256;
    if (tcap > 0 && tb > tcap) tb = tcap;
    // candidates per chunk: the longest element this layout can produce (a record with a
    // timestamp: 4 + 1 + 8 + vbytes; the other tags are at most 33 bytes)
    const bool wide = 13 + L.vbytes > 64;
#define NB_LAUNCH(NL)                                                                                              \
    hipLaunchKernelGGL(k_nb_walk<NL>, dim3((unsigned)gb), dim3(256), 0, s, buf, nbytes, nch, L.vbytes, exits, cnt, \
                       conv, sync, d_st);                                                                          \
    hipLaunchKernelGGL(k_nb_tail<NL>, dim3((unsigned)tb), dim3(256), 0, s, buf, nbytes, nch,                       \
                       L.vbytes, sync, conv, tcnt, tmask);                                                         \
    hipLaunchKernelGGL(k_nb_resolve<NL>, dim3((unsigned)nblk), dim3(kNbScanBlock), 0, s, nbytes, nch, exits, cnt,  \
                       conv, sync, tcnt, entry, offs, btot, d_st);                                                 \
    hipLaunchKernelGGL(k_nb_scan, dim3(1), dim3(1024), 0, s, nblk, btot, d_st);                                    \
    hipLaunchKernelGGL(k_nb_decode<NL>, dim3((unsigned)gb), dim3(256), 0, s, buf, nbytes, nch, L, entry, offs, btot, \
                       sync, tmask, key, ts, val, rec_cap, wm_pos, wm_val, wm_cap, d_st)
    if (wide) {
        NB_LAUNCH(GW_MAX_ELEMENT);
    } else {
        NB_LAUNCH(64);
    }
#undef NB_LAUNCH
    return hipGetLastError();
}

}  // namespace gw
