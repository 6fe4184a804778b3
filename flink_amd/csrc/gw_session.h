// gw_session.h — host interface of the event-time session-window path (gw_session.hip).
#pragma once
#include <functional>
#include <string>
#include <vector>

#include "gw_device.h"

namespace gw {

struct SessionState;

int session_create(SessionState*& s, const gw_config& cfg, int64_t cap, hipStream_t stream, DevStatus* unused,
                   std::string& why);
void session_destroy(SessionState* s);
int session_ingest(SessionState* s, int64_t n, const int64_t* key, const int64_t* ts, const int64_t* val,
                   int64_t wm, std::string& err);
int session_fire(SessionState* s, int64_t wm, int64_t* fired, std::string& err);
void session_rows(SessionState* s, int64_t** k, int64_t** st, int64_t** en, int64_t** r, int64_t* total);
int session_refresh(SessionState* s, std::string& err);
// State of key groups [kg_lo, kg_hi] as entries of session_entry_words() int64 each:
// sessions (key, start, end, a0, a1, fired) per in-flight session; count windows (key, element
// count, ring of pane accumulators) per key.
int session_entry_words(SessionState* s);
// hash_of: the Java hashCode of a key (empty: Long.hashCode).
int session_collect(SessionState* s, int32_t kg_lo, int32_t kg_hi, std::vector<int64_t>& ent,
                    std::vector<int32_t>& kgs, std::string& err,
                    const std::function<int32_t(int64_t)>& hash_of = nullptr);
// Insert n entries of session_entry_words() int64 (as session_collect writes them).
int session_restore(SessionState* s, const int64_t* ent, int64_t n, std::string& err);
int session_clear_rows(SessionState* s, std::string& err);
int64_t session_late(SessionState* s);
int session_pending_late(SessionState* s, int64_t* n, std::string& err);
int session_drain_late(SessionState* s, int64_t* key, int64_t* ts, int64_t* val, int64_t cap, int64_t* n,
                       std::string& err);
void session_stats(SessionState* s, gw_stats* out);
void session_enable_timing(SessionState* s, bool on);
int session_kernel_time(SessionState* s, int which, double* ms, int64_t* launches);

}  // namespace gw
