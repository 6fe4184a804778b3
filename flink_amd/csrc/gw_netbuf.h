// gw_netbuf.h — network-buffer decode (gw_netbuf.hip): layout, status, launcher.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpuwin.h"

namespace gw {

#ifndef GW_NB_CHUNK
#define GW_NB_CHUNK 1024
#endif
constexpr int kNbChunk = GW_NB_CHUNK;  // bytes per wave in the chain walk

// The record value layout reduced to what the decoder needs (validated on the host).
struct NbLayout {
    int32_t vbytes;    // serialized value bytes (sum of the field widths)
    int32_t key_off;   // byte offset of the Long key field in the value
    int32_t val_off;   // byte offset of the aggregated field
    int32_t val_type;  // its type code ('J', 'D', ...), 0 = none (COUNT)
};

struct NbStatus {
    unsigned long long corrupt;      // unknown tag / length that does not match the element
    unsigned long long unsupported;  // an element longer than GW_MAX_ELEMENT
    unsigned long long full;         // rec_cap / wm_cap exceeded
    unsigned long long skipped;      // latency markers, stream status, record attributes
    long long consumed;              // bytes up to the end of the last complete element
    long long records, watermarks;
    unsigned long long walkback;     // chunk steps k_nb_resolve walked back over non-converged chunks
    unsigned long long fallback;     // chunks whose candidates disagreed after the sync window
};

inline int nb_field_width(char t) {
    switch (t) {
    case 'J': case 'D': return 8;
    case 'I': case 'F': return 4;
    case 'S': return 2;
    case 'B': case 'Z': return 1;
    default: return -1;
    }
}

int64_t nb_scratch_bytes(int64_t nbytes);
hipError_t launch_nb_decode(const uint8_t* buf, int64_t nbytes, const NbLayout& L, int64_t* key, int64_t* ts,
                            int64_t* val, int64_t rec_cap, int64_t* wm_pos, int64_t* wm_val, int64_t wm_cap,
                            void* scratch, NbStatus* d_st, hipStream_t s);

}  // namespace gw
