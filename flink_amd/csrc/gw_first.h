// gw_first.h — first-element rows (GW_FLAG_FIRST_ELEMENT): the device side of joining a
// window's aggregate row with the payload of its first element (gw_first.hip).
#pragma once
#include "gw_device.h"

namespace gw {
// Scratch bytes fe_join needs for n rows.
size_t fe_join_scratch_bytes(int64_t n);
// Rows A (the aggregate) and B (MIN of the arrival sequence) hold the same (key, window) set
// in different orders.  Writes A's rows sorted by (key, start) into o_* and, per row, the
// payload log entry of B's minimum sequence: o_pay[i] = log[(seq - log_base) mod log_cap].
hipError_t fe_join(int64_t n, const int64_t* a_key, const int64_t* a_start, const int64_t* a_end,
                   const int64_t* a_res, const int64_t* b_key, const int64_t* b_start, const int64_t* b_res,
                   const int64_t* log, int64_t log_base, int64_t log_cap, int64_t* o_key, int64_t* o_start,
                   int64_t* o_end, int64_t* o_res, int64_t* o_pay, void* scratch, size_t scratch_bytes,
                   int32_t* d_bad, hipStream_t s);
// d[i] = base + i (the arrival sequence of a batch's records).
hipError_t fe_iota64(int64_t* d, int64_t n, int64_t base, hipStream_t s);
// out[0] = max(out[0], max over ts[0..n)) (a batch's largest timestamp, for the log's retention).
hipError_t fe_max_ts(const int64_t* ts, int64_t n, int64_t* out, hipStream_t s);
// Copy the live sequences [base, end) of a log ring of ocap words into one of ncap words.
hipError_t fe_log_regrow(const int64_t* o, int64_t ocap, int64_t* d, int64_t ncap, int64_t base, int64_t end,
                         hipStream_t s);
// out[i] = log[seq[i] mod cap] (the payloads of a snapshot's first elements).
hipError_t fe_log_gather(const int64_t* log, int64_t cap, const int64_t* seq, int64_t n, int64_t* out, hipStream_t s);
// Append n payload words at log position pos (a ring of cap words).
hipError_t fe_log_append(int64_t* log, int64_t cap, int64_t pos, const int64_t* src, int64_t n, hipStream_t s);
// minBy / maxBy (GW_FLAG_BY_FIELD): scratch bytes fe_by_select needs for n rows.
size_t fe_by_scratch_bytes(int64_t n);
// For each of the n rows (key, start, res = the window's MIN / MAX of the field), the sequence of
// the element it stands for: the first (last) live log record [log_base, log_end) of the row's
// key and window whose field equals res.  The log holds 4 columns of log_cap words (payload, key,
// ts, field); records below restored_end are restored elements of the window starting at their
// ts.  o_seq / o_pay (either may be null) get the sequence and its payload; *d_bad |= 2 when a
// row has no element in the log.
// is_max: res is the window's MAX (maxBy), else its MIN (minBy): lets the scan skip records
// that cannot equal any row of their bucket.
hipError_t fe_by_select(int64_t n, const int64_t* key, const int64_t* start, const int64_t* res, const int64_t* log,
                        int64_t log_cap, int64_t log_base, int64_t log_end, int64_t restored_end, int64_t offset,
                        int64_t slide, int64_t size, bool last, bool f64, bool is_max, int64_t* o_seq, int64_t* o_pay,
                        void* scratch, size_t scratch_bytes, int32_t* d_bad, hipStream_t s);
}  // namespace gw
