/*
 * flink_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A CPU restatement of Apache Flink's keyed event-time window operator
 * (WindowOperator + HashMapStateBackend + EventTimeTrigger + MergingWindowSet),
 * used as the parity oracle for libgpuwin.so and as the CPU baseline in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product path (flink_amd/, libgpuwin.so) never does.
 *
 * It follows the reference algorithm record by record — one state entry per
 * (key, window), a deduplicated timer heap, per-key merging window sets —
 * NOT the GPU's pane/slice design, so the two are independent restatements.
 *
 * Pinning: tests/test_oracle_golden.py checks it against every golden vector
 * transcribed from the reference's own tests (tests/golden/).
 */
#ifndef FLINK_ORACLE_H
#define FLINK_ORACLE_H
#include <stdint.h>
#include "../include/gpuwin.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wo_op wo_op;

/* primitives (MathUtils / KeyGroupRangeAssignment / TimeWindow / JDK hashCode) */
int32_t wo_murmur_hash(int32_t code);
int32_t wo_bit_mix(int32_t in);
int32_t wo_long_to_int_with_bit_mixing(int64_t in);
int32_t wo_long_hash(int64_t v);
int32_t wo_string_hash(const uint16_t* utf16, int64_t n);
int32_t wo_assign_to_key_group(int32_t key_hash, int32_t max_parallelism);
int32_t wo_operator_index_for_key_group(int32_t max_p, int32_t p, int32_t kg);
void    wo_key_group_range(int32_t max_p, int32_t p, int32_t idx, int32_t* start, int32_t* end);
int32_t wo_default_max_parallelism(int32_t p);
int64_t wo_window_start_with_offset(int64_t ts, int64_t offset, int64_t size);
/* Windows of one record; returns count (<= cap) or a negative GW_E_* code. */
int     wo_assign_windows(const gw_config* cfg, int64_t ts, int64_t* start, int64_t* end, int cap);
/* TimeWindow.mergeWindows on n windows: writes, per input window, the index of its
 * merge group (groups numbered in sort order) and per group the cover window.
 * Returns the number of groups. */
int     wo_merge_windows(int n, const int64_t* start, const int64_t* end,
                         int32_t* group_of, int64_t* gstart, int64_t* gend);

/* operator */
int     wo_validate(const gw_config* cfg);
wo_op*  wo_create(const gw_config* cfg);
void    wo_destroy(wo_op* op);
int     wo_process_element(wo_op* op, int64_t key, int64_t ts, int64_t value_bits);
int     wo_process_batch(wo_op* op, int64_t n, const int64_t* key, const int64_t* ts,
                         const int64_t* value_bits);
int     wo_process_watermark(wo_op* op, int64_t wm);
/* key.hashCode() of keys the caller maps to int64 ids (String, Integer, ... keys): their key
 * group, and the key hash a snapshot entry carries, follow it (default Long.hashCode). */
int     wo_set_key_hashes(wo_op* op, int64_t n, const int64_t* key, const int32_t* hash);
int64_t wo_output_count(const wo_op* op);
/* Copies and removes up to cap rows. result is 8 bytes per row (int64 or double). */
int64_t wo_drain(wo_op* op, int64_t* key, int64_t* start, int64_t* end, int64_t* result_bits,
                 int64_t cap);
/* wo_drain plus q[i]: the arrival number (0-based over every wo_process_element call) of the
 * element a minBy / maxBy row stands for (GW_FLAG_BY_FIELD; tumbling / sliding windows). */
int64_t wo_drain_seq(wo_op* op, int64_t* key, int64_t* start, int64_t* end, int64_t* result_bits, int64_t* q,
                     int64_t cap);
int64_t wo_late_dropped(const wo_op* op);
/* The arrival number of the next element (wo_drain_seq's q): a restored operator continues the
 * numbering of the one that wrote the snapshot. */
void    wo_set_arrival(wo_op* op, int64_t next);
/* Late-data side output (config flag GW_FLAG_LATE_SIDE_OUTPUT): the skipped late elements. */
int64_t wo_late_output_count(const wo_op* op);
int64_t wo_drain_late(wo_op* op, int64_t* key, int64_t* ts, int64_t* value_bits, int64_t cap);
int64_t wo_current_watermark(const wo_op* op);
int64_t wo_state_entries(const wo_op* op);
int64_t wo_timer_count(const wo_op* op);
int64_t wo_session_merges(const wo_op* op);
const char* wo_last_error(const wo_op* op);

/* Keyed state of key groups [kg_lo, kg_hi] in the heap backend's per-key-group layout
 * (blob version 4 of include/gpuwin.h gw_snapshot).  Returns the size; writes the blob
 * when cap is large enough.  wo_restore reads one blob back (state, merging window sets,
 * timers); the watermark is not part of it. */
int64_t wo_snapshot(wo_op* op, int32_t kg_lo, int32_t kg_hi, uint8_t* buf, int64_t cap);
int     wo_restore(wo_op* op, const uint8_t* buf, int64_t len);
int     wo_acc_bytes(int agg);

/* A stand-alone MergingWindowSet of session windows (MergingWindowSet.java:77-224), the unit
 * MergingWindowSetTest drives: wo_mws_add = addWindow with a recording MergeFunction (res[2]
 * = the result window; info = merged?, mergeResult (2), stateWindowResult (2), n sources, the
 * merged windows (2 each), n state windows, the merged state windows (2 each)).
 * wo_mws_state_window = getStateWindow (returns 0 for null); wo_mws_retire = retireWindow
 * (GW_E_STATE when absent); wo_mws_put = the restore from the ListState; wo_mws_list = the
 * persisted (window, state window) list, returns its length. */
typedef struct wo_mws wo_mws;
wo_mws* wo_mws_create(void);
void    wo_mws_destroy(wo_mws* w);
int     wo_mws_add(wo_mws* w, int64_t start, int64_t end, int64_t* res, int64_t* info);
int     wo_mws_state_window(const wo_mws* w, int64_t start, int64_t end, int64_t* out);
int     wo_mws_retire(wo_mws* w, int64_t start, int64_t end);
void    wo_mws_put(wo_mws* w, int64_t start, int64_t end, int64_t state_start, int64_t state_end);
int     wo_mws_list(const wo_mws* w, int64_t* out, int cap);

/* Multi-threaded CPU baseline: `threads` operator instances, each owning the key
 * groups of one subtask (computeKeyGroupRangeForOperatorIndex), like a Flink job
 * at parallelism = threads.  Runs the whole stream: batches of batch_len records,
 * each followed by watermark wm[b]; then MAX_WATERMARK.  Returns rows fired and
 * writes the wall time to *seconds. */
int64_t wo_run_parallel(const gw_config* cfg, int threads, int64_t n_batches,
                        const int64_t* batch_len, const int64_t* wm,
                        const int64_t* key, const int64_t* ts, const int64_t* value_bits,
                        int64_t* checksum, double* seconds);
/* The same without the final MAX_WATERMARK: only the stream's own watermarks (the cadence a
 * benchmark's timed steps run at). */
int64_t wo_run_parallel_stream(const gw_config* cfg, int threads, int64_t n_batches,
                               const int64_t* batch_len, const int64_t* wm,
                               const int64_t* key, const int64_t* ts, const int64_t* value_bits,
                               int64_t* checksum, double* seconds);
/* The same keeping every fired row (key, start, end, result bits, watermark index b; nb for
 * the final MAX_WATERMARK) in caller arrays of cap rows; GW_E_OUTPUT_FULL beyond cap. */
int64_t wo_run_parallel_rows(const gw_config* cfg, int threads, int64_t n_batches,
                             const int64_t* batch_len, const int64_t* wm,
                             const int64_t* key, const int64_t* ts, const int64_t* value_bits,
                             int64_t cap, int64_t* o_key, int64_t* o_start, int64_t* o_end, int64_t* o_res,
                             int32_t* o_wm, double* seconds);
/* The same, per watermark: wm_rows[b] / wm_cs[b] for b = 0..n_batches (the last entry is
 * the final MAX_WATERMARK) hold the rows that watermark fired over all subtasks and the
 * sum of their row hashes, (key * 0x9e3779b97f4a7c15) ^ (start * 31) ^ (end * 17) ^ result
 * mod 2^64. */
int64_t wo_run_parallel_wm(const gw_config* cfg, int threads, int64_t n_batches,
                           const int64_t* batch_len, const int64_t* wm,
                           const int64_t* key, const int64_t* ts, const int64_t* value_bits,
                           int64_t* wm_rows, int64_t* wm_cs, double* seconds);

/* Sequential decode of one input channel's serialized stream elements (the GPU's
 * gw_decode_serialized restated record by record). */
int     wo_decode_stream(const uint8_t* buf, int64_t nbytes, const gw_record_layout* lay,
                         int64_t* key, int64_t* ts, int64_t* value_bits, int64_t rec_cap,
                         int64_t* wm_pos, int64_t* wm_val, int64_t wm_cap, gw_decode_result* out);

#ifdef __cplusplus
}
#endif
#endif
