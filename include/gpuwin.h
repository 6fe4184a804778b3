/*
 * gpuwin.h — C ABI of libgpuwin.so, the MI355X-native keyed event-time window
 * aggregation operator (a drop-in for Flink's WindowOperator on the
 * keyBy().window(...).aggregate/reduce path).
 *
 * Plain C types only: pointers, sizes, int64 timestamps. No torch, no C++.
 * Every entry point returns an int status (0 = GW_OK, negative = error) and
 * never lets a C++ exception cross the boundary; gw_last_error() explains a
 * failure.  The JVM shim turns a negative status into an
 * Exception, which is exactly how the reference operator fails its task
 * ("Any exception from processElement or onEventTime fails the
 * task").
 *
 * Reference slot replaced (paths relative to the Flink tree,
 * RS/ = flink-runtime/src/main/java/org/apache/flink/streaming/):
 *   gw_create            WindowOperatorFactory.createStreamOperator
 *                          (RS/runtime/operators/windowing/WindowOperatorFactory.java:96-99)
 *                        + WindowOperator.open (WindowOperator.java:226-281)
 *   gw_ingest            WindowOperator.processElement, batched over all records
 *                        between two watermarks (WindowOperator.java:293-447;
 *                        per-record dispatch OneInputStreamTask.java:249-252)
 *   gw_advance_watermark AbstractStreamOperator.processWatermark ->
 *                        InternalTimerServiceImpl.tryAdvanceWatermark ->
 *                        WindowOperator.onEventTime
 *                        (AbstractStreamOperator.java:690-703,
 *                         InternalTimerServiceImpl.java:328-347,
 *                         WindowOperator.java:450-494)
 *   gw_drain             TimestampedCollector / Output.collect of the fired rows
 *                        (WindowOperator.emitWindowContents :575-580)
 *   gw_late_dropped      WindowOperator.numLateRecordsDropped (:144,229)
 *   gw_destroy           WindowOperator.close / dispose
 *   gw_java_long_hash,
 *   gw_murmur_hash,
 *   gw_key_group_*       KeyGroupRangeAssignment (flink-runtime/.../runtime/state/
 *                        KeyGroupRangeAssignment.java:50-147), MathUtils.murmurHash
 *                        (flink-core/.../util/MathUtils.java:137-201)
 *   gw_partition_device  KeyGroupStreamPartitioner.selectChannel
 *                        (RS/runtime/partitioner/KeyGroupStreamPartitioner.java:55-64)
 *                        feeding the RCCL all-to-all that replaces the Netty keyBy shuffle
 */
#ifndef GPUWIN_H
#define GPUWIN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GW_ABI_VERSION 3

/* ---- status codes -------------------------------------------------------- */
#define GW_OK              0
#define GW_E_INVALID      -1  /* bad argument / config (Flink: IllegalArgumentException)      */
#define GW_E_UNSUPPORTED  -2  /* valid in Flink, not (yet) on the GPU path                   */
#define GW_E_DEVICE       -3  /* HIP runtime error                                            */
#define GW_E_OOM          -4  /* device or host allocation failed                             */
#define GW_E_OUTPUT_FULL  -5  /* more fired rows pending: call gw_drain again                 */
#define GW_E_NO_TIMESTAMP -6  /* record carries Long.MIN_VALUE (assigners throw RuntimeException) */
#define GW_E_RANGE        -7  /* window bounds overflow int64                                 */
#define GW_E_STATE        -8  /* illegal call sequence / merge into the past                  */

/* ---- configuration ------------------------------------------------------- */
typedef enum gw_assigner {
    GW_TUMBLING = 0, /* TumblingEventTimeWindows.of(size, offset)  (stagger ALIGNED)   */
    GW_SLIDING  = 1, /* SlidingEventTimeWindows.of(size, slide, offset)                */
    GW_SESSION  = 2, /* EventTimeSessionWindows.withGap(gap)                           */
    /* Count windows over GlobalWindows, per key in arrival order;
     * timestamps, watermarks and allowed lateness play no part (GlobalWindows is not an
     * event-time assigner).  A row is (key, first element ordinal, end ordinal, result):
     * the window holds the key's elements [start, end) in arrival order, counted from 0.
     * Rows are produced by gw_ingest* itself (CountTrigger fires on the element). */
    GW_COUNT_TUMBLING = 3, /* KeyedStream.countWindow(size): PurgingTrigger(CountTrigger(size))
                              (RS/api/datastream/KeyedStream.java:676-678)                  */
    GW_COUNT_SLIDING  = 4  /* KeyedStream.countWindow(size, slide): CountEvictor(size) +
                              CountTrigger(slide) (KeyedStream.java:686-690)                */
} gw_assigner;

typedef enum gw_trigger {
    GW_EVENT_TIME_TRIGGER         = 0, /* EventTimeTrigger.create()                   */
    GW_PURGING_EVENT_TIME_TRIGGER = 1  /* PurgingTrigger.of(EventTimeTrigger.create()) */
} gw_trigger;

/* The closed set of aggregate functions of the path.
 * Result column type: int64 for COUNT/SUM_I64/MIN_I64/MAX_I64/SUM_I32 (sign-extended
 * Java int), IEEE double for SUM_F64/MIN_F64/MAX_F64/AVG_I64/AVG_F64. */
typedef enum gw_agg {
    GW_COUNT   = 0, /* AggregateFunction<T, Long, Long> counting records           */
    GW_SUM_I64 = 1, /* WindowedStream.sum on a Long field (Java wrap-around)        */
    GW_SUM_F64 = 2, /* WindowedStream.sum on a Double field                         */
    GW_MIN_I64 = 3, /* WindowedStream.min on a Long field                           */
    GW_MAX_I64 = 4, /* WindowedStream.max on a Long field                           */
    GW_MIN_F64 = 5, /* WindowedStream.min on a Double field (Double.compareTo order) */
    GW_MAX_F64 = 6, /* WindowedStream.max on a Double field                         */
    GW_AVG_I64 = 7, /* AverageAggregate: acc (long sum, long count) -> (double)sum/count */
    GW_AVG_F64 = 8, /* acc (double sum, long count) -> sum/count                    */
    GW_SUM_I32 = 9  /* WindowedStream.sum on an Integer field (int32 wrap-around)   */
} gw_agg;

typedef struct gw_config {
    int32_t assigner;         /* gw_assigner                                          */
    int32_t trigger;          /* gw_trigger                                           */
    int64_t size;             /* tumbling/sliding window size, ms                     */
    int64_t slide;            /* sliding slide, ms (ignored for tumbling)             */
    int64_t offset;           /* window offset, ms                                    */
    int64_t gap;              /* session gap, ms                                      */
    int64_t allowed_lateness; /* WindowedStream.allowedLateness, ms (>= 0)            */
    int32_t agg;              /* gw_agg                                               */
    int32_t max_parallelism;  /* number of key groups (0 -> 128)                      */
    int32_t parallelism;      /* operator parallelism (0 -> 1)                        */
    int32_t operator_index;   /* this subtask                                         */
    int32_t device;           /* HIP device ordinal                                   */
    int32_t flags;            /* GW_FLAG_*                                            */
    int64_t capacity_hint;    /* expected live keys (sizes the HBM state table)       */
    int64_t max_batch;        /* records per ingest call (sizes staging), 0 -> 1<<20  */
} gw_config;

#define GW_FLAG_FORCE_LDS_PREAGG   1 /* always pre-aggregate in LDS before the HBM RMW  */
#define GW_FLAG_NO_LDS_PREAGG      2 /* never pre-aggregate in LDS                       */
#define GW_FLAG_CHECK_KEY_GROUPS   4 /* reject keys outside this subtask's key groups    */
#define GW_FLAG_FORCE_REGION       8 /* always use the region-bucketed ingest path      */
#define GW_FLAG_NO_REGION         16 /* never use the region-bucketed ingest path       */
#define GW_FLAG_NO_BUFFER         32 /* region path: apply every batch at once instead of
                                        buffering pass-1 segments until the next fire    */
#define GW_FLAG_LATE_SIDE_OUTPUT  64 /* WindowedStream.sideOutputLateData: late records go to
                                        gw_drain_late instead of numLateRecordsDropped    */
#define GW_FLAG_NO_NARROW        256 /* region path: never narrow records (compact or wide only) */
#define GW_FLAG_FIRST_ELEMENT    128 /* positional sum/min/max (WindowedStream.sum(i) etc.):
                                        records carry a 64-bit payload (the tuple's other
                                        fields, packed by the caller) and every row carries the
                                        payload of its window's first element in arrival
                                        order (gw_ingest_payload*, gw_drain_payload);
                                        tumbling / sliding windows with EventTimeTrigger    */
#define GW_FLAG_BY_FIELD       512 /* minBy / maxBy (WindowedStream.minBy(i, first) etc.,
                                        WindowedStream.java:725-771; ComparableAggregator
                                        byAggregate, ComparableAggregator.java:88-95): with
                                        GW_MIN_* / GW_MAX_*, every row carries the payload of
                                        the window's element whose field is the minimum /
                                        maximum, the first of equal ones in arrival order
                                        (implies GW_FLAG_FIRST_ELEMENT's payload ingest/drain) */
#define GW_FLAG_BY_LAST       1024 /* with GW_FLAG_BY_FIELD: the last of equal ones
                                        (minBy(i, false)); needs allowed lateness 0         */

typedef struct gw_handle gw_handle;

/* Per-operator counters (Flink: numRecordsIn, numLateRecordsDropped, numFiredTimers). */
typedef struct gw_stats {
    int64_t events_in;        /* records handed to gw_ingest*                      */
    int64_t late_dropped;     /* numLateRecordsDropped                             */
    int64_t rows_fired;       /* fired (key, window) rows so far                   */
    int64_t live_keys;        /* occupied state-table slots                        */
    int64_t table_capacity;   /* state-table slots                                 */
    int64_t table_bytes;      /* HBM bytes of the state table                      */
    int64_t deferred;         /* partial aggregates parked outside the pane ring   */
    int64_t batches;          /* ingest calls                                      */
    int64_t fires;            /* fire passes launched                              */
    int64_t rehashes;         /* table growths                                     */
    int64_t preagg_batches;   /* batches that used the LDS pre-aggregation kernel  */
    int64_t session_merges;   /* sessions merged away (M_b)                        */
    int64_t applies;          /* region pass-2 + apply launches (buffer flushes)   */
    int64_t region_format;    /* record format of the last region flush window: 0 wide,
                                 1 compact (hash word + 32-bit value), 2 narrow (32-bit
                                 key + 28-bit value; 4 B for COUNT); -1 none yet       */
    int64_t session_punted;   /* session records whose key found no free slot in the main
                                 table: replayed after the table grew                    */
    int64_t session_slow;     /* reserved (0): the removed bucketed session ingest's
                                 general-path count                                      */
} gw_stats;

/* ---- lifecycle ------------------------------------------------------------ */
int  gw_create(const gw_config* cfg, gw_handle** out);
int  gw_destroy(gw_handle* h);
/* Last error text of h (or of the last failed gw_create when h == NULL). */
const char* gw_last_error(const gw_handle* h);
int  gw_abi_version(void);

/* ---- data path ------------------------------------------------------------ */
/* Host columns: key[n], ts[n], value[n] (8 bytes each: int64 or IEEE double per agg;
 * value may be NULL for GW_COUNT).  key_hash[n] (Java key.hashCode()) may be NULL:
 * the key group is then computed from Long.hashCode(key).  Buffers are reusable as
 * soon as the call returns.  All records of one call see the same current
 * watermark (the one last passed to gw_advance_watermark), which is exactly what a
 * Flink operator sees for the records between two watermarks. */
int  gw_ingest(gw_handle* h, int64_t n, const int64_t* key, const int32_t* key_hash,
               const int64_t* ts, const void* value);
/* Library-owned pinned column slots for callers that build a batch in place (the JVM operator
 * writes each record's fields straight into them as direct ByteBuffers, so no copy precedes the
 * PCIe transfer).  gw_stage_alloc: `slots` slots of `cap` records.  gw_stage_columns: slot's
 * key / key_hash / ts / value columns (any pointer may be NULL), once the slot's previous
 * transfer has read it.  gw_ingest_stage: the slot's first n records, as gw_ingest would take
 * them (cols: GW_STAGE_VALUE and / or GW_STAGE_KEY_HASH); the transfer runs on a copy stream
 * into one of three device buffers used in turn, so it overlaps the previous batches' kernels.  The
 * slot may be refilled after the next gw_stage_columns on it returns.  Not for composite or
 * first-element handles (GW_E_UNSUPPORTED). */
#define GW_STAGE_VALUE    1
#define GW_STAGE_KEY_HASH 2
int  gw_stage_alloc(gw_handle* h, int32_t slots, int64_t cap);
int  gw_stage_columns(gw_handle* h, int32_t slot, int64_t** key, int32_t** key_hash, int64_t** ts,
                      int64_t** value);
int  gw_ingest_stage(gw_handle* h, int32_t slot, int64_t n, int32_t cols);
/* Send a filled slot's first n records over PCIe ahead of its gw_ingest_stage (into the next of
 * the three device buffers, once the ingest that last read it is done), e.g. batches b+1 and b+2
 * while batch b is fired and its rows drained.  At most two batches ahead; the gw_ingest_stage
 * calls must name the sent slots, n and cols in the order they were sent (GW_E_STATE otherwise). */
int  gw_stage_send(gw_handle* h, int32_t slot, int64_t n, int32_t cols);
/* Same, with the columns already resident in device memory (d_* are device
 * pointers).  `stream` is the hipStream_t the inputs were produced on (NULL = the
 * default stream).  The handle's stream (gw_stream) reads them after that stream's
 * pending work, and the producer stream is made to wait for those reads, so the caller
 * may reuse or free the columns in stream order on the producer stream (e.g. a PyTorch
 * caching allocator) without further synchronisation. */
int  gw_ingest_device(gw_handle* h, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                      const int64_t* d_ts, const void* d_value, void* stream);
/* Advance event time to wm: fire every window whose maxTimestamp (end-1) <= wm,
 * purge its state, and append the fired rows to the output.  *rows_fired (may be
 * NULL) receives the number of rows this call produced.  Watermarks that do not
 * advance are ignored, as in InternalTimerServiceImpl.tryAdvanceWatermark. */
int  gw_advance_watermark(gw_handle* h, int64_t wm, int64_t* rows_fired);
/* Apply every buffered record to the window state now.  The region path buffers
 * pass-1 segments of several watermark batches and applies them before the next fire
 * by itself; gw_flush makes the state exact at any point, as a snapshot needs
 * (StreamOperator.prepareSnapshotPreBarrier, RS/api/operators/StreamOperator.java:122). */
int  gw_flush(gw_handle* h);
/* ---- checkpoint / restore ------------------------------------------------ */
/* Snapshot of the window state of key groups [kg_lo, kg_hi] (buffered records are
 * applied first).  Replaces the keyed-state part of StreamOperator.snapshotState
 * (RS/api/operators/StreamOperator.java:131) in the heap backend's per-key-group layout
 * (HeapSnapshotStrategy.java:97-154).  The blob is a 96-byte header (magic "GWS1",
 * version, window, aggregate, max parallelism, key-group range, flags), int64
 * kg_offsets[kg_hi - kg_lo + 2], then per key group:
 *   version 4 (tumbling / sliding windows, also under allowed lateness and PurgingTrigger;
 *   big-endian like DataOutputView): be32 n + n "window-contents" entries
 *   (window.start, window.end, key, [be32 key hash,] state) as
 *   CopyOnWriteStateMapSnapshot.writeState writes them (:127-149; one entry per (key,
 *   window) holding state: not fired, or fired and kept until its cleanup time), be32 0
 *   (no merging window set), be32 t + t event-time timers (flipSignBit(ts), key, start,
 *   end) as TimerSerializer.serialize writes them (:147-152; the window's maxTimestamp
 *   and, under lateness, its cleanup time);
 *   version 4 (session windows): the same three sections -- be32 n + n "window-contents"
 *   entries (state window, key, [be32 key hash,] state) of the sessions holding state (a
 *   session fired under PurgingTrigger holds none), be32 m + m "merging-window-set" records
 *   (key, [be32 key hash,] be32 c, c x (window, state window)) as MergingWindowSet.persist
 *   writes its ListState (:99-106), be32 t + t timers (maxTimestamp while a session has not
 *   fired; its cleanup time under allowed lateness).  libgpuwin names each session as its own
 *   state window; a restore takes any state window the set names (the reference keeps a
 *   merged session's state under one of its original windows, MergingWindowSet.java:188-201);
 *   version 3 (count windows): per key (key, element count, ring of count-pane
 *   accumulators): the CountTrigger count and the evicting operator's window contents.
 * Keys fed with a key_hash column (String, Integer, ... keys as caller ids) are filed
 * under the key group of that hash (KeyGroupRangeAssignment.java:63-66), and the blob
 * carries each entry's key hash (header flags bit 0: a be32 after the key of every
 * version-4 entry and merging-window-set record, one more int64 word per entry in version 3).  A window-class composite writes
 * its classes' entries merged per key group.  Two calls: buf == NULL returns the size in
 * *len; then a buffer of cap >= *len. */
int  gw_snapshot(gw_handle* h, int32_t kg_lo, int32_t kg_hi, void* buf, int64_t cap, int64_t* len);
/* Restore one snapshot blob (call once per key-group range, e.g. after rescaling) into a
 * handle with the same assigner, aggregate and max parallelism
 * (StreamOperator.initializeState, StreamOperator.java:139).  The watermark is not part
 * of the state: like Flink after a restore it starts at Long.MIN_VALUE. */
int  gw_restore(gw_handle* h, const void* buf, int64_t len);

/* The part of a gw_snapshot blob that belongs to key group kg, as a blob of its own (what
 * GpuWindowOperator writes per key group into the raw keyed state stream, like the heap
 * backend's per-key-group write, HeapSnapshotStrategy.java:97-154).  Pure host code; any
 * blob version.  Two calls as gw_snapshot: out == NULL returns the size in *out_len.
 * GW_E_INVALID for a corrupt blob or kg outside its key-group range (gw_last_error(NULL)). */
int  gw_snapshot_slice(const void* blob, int64_t len, int32_t kg, void* out, int64_t cap, int64_t* out_len);

/* The distinct keys a blob's entries and timers name, ascending, into keys[cap]; *n gets
 * their number (keys == NULL: only the count).  With gw_snapshot_remap_keys this is what a
 * caller that maps its keys to int64 ids (GpuWindowOperator<IN, K> for non-Long K) needs
 * to write the real keys beside the blob (through the key serializer) and to restore them
 * under the ids of another process.  Pure host code; GW_E_INVALID for a corrupt blob. */
int  gw_snapshot_keys(const void* blob, int64_t len, int64_t* keys, int64_t cap, int64_t* n);
/* Rewrite in place every key of the blob found in from[0..n) (ascending) to the matching
 * to[i]; key hashes stay.  GW_E_INVALID for a corrupt blob or unsorted from[]. */
int  gw_snapshot_remap_keys(void* blob, int64_t len, const int64_t* from, const int64_t* to, int64_t n);
/* First-element handles (GW_FLAG_FIRST_ELEMENT): their blob's version-4 entries end with the
 * be64 payload of the window's first element (header flags bit 1).  gw_snapshot_payloads
 * lists the distinct payloads ascending (payloads == NULL: only the count) and the latest
 * window end among the entries -- what the caller needs to write the elements beside the
 * blob and to keep them after a restore until those windows are cleaned;
 * gw_snapshot_remap_payloads rewrites them to a restoring process's own ids. */
int  gw_snapshot_payloads(const void* blob, int64_t len, int64_t* payloads, int64_t cap, int64_t* n,
                          int64_t* max_window_end);
int  gw_snapshot_remap_payloads(void* blob, int64_t len, const int64_t* from, const int64_t* to, int64_t n);

/* ---- network-buffer ingest ----------------------------- */
/* Layout of the record value: a Flink Tuple of fixed-width fields as TupleSerializer
 * writes them (fields in order, no null markers; flink-core/.../api/java/typeutils/
 * runtime/TupleSerializer.java:139-145), each field big-endian as DataOutputView
 * writes it (LongSerializer.serialize = writeLong, DoubleSerializer = writeDouble,
 * IntSerializer = writeInt, ...).  Type codes are JVM descriptors:
 *   'J' long, 'D' double, 'I' int, 'F' float, 'S' short, 'B' byte, 'Z' boolean. */
#define GW_MAX_FIELDS 8
typedef struct gw_record_layout {
    int32_t nfields;               /* fields of the Tuple (1..GW_MAX_FIELDS)             */
    int32_t key_field;             /* index of the Long key field (keyBy(t -> t.fN))     */
    int32_t value_field;           /* index of the aggregated field; -1 for GW_COUNT     */
    char    types[GW_MAX_FIELDS];  /* type code per field                                */
} gw_record_layout;

/* Result of decoding one input channel's bytes. */
typedef struct gw_decode_result {
    int64_t records;    /* StreamRecords decoded (columns written)                         */
    int64_t watermarks; /* Watermark elements (wm_pos/wm_val written)                      */
    int64_t consumed;   /* bytes up to the end of the last complete element; the caller
                           keeps the rest and prepends it to the next call (a record
                           spanning network buffers, SpanningWrapper)                      */
    int64_t skipped;    /* latency markers, stream status and record attributes            */
} gw_decode_result;

/* Decode the serialized stream elements of one input channel on the device.  The bytes
 * are the concatenated payloads of the channel's network buffers: per element a 4-byte
 * big-endian length, then StreamElementSerializer's tag and body
 * (RecordWriter.serializeRecord, flink-runtime/.../io/network/api/writer/
 * RecordWriter.java:144-156; StreamElementSerializer.serialize/deserialize,
 * RS/runtime/streamrecord/StreamElementSerializer.java:163-225).  Records go to the
 * columns (key, timestamp, value as 8-byte int64 / IEEE double bits; a record without
 * timestamp gets Long.MIN_VALUE), watermarks to (wm_pos = number of records before it,
 * wm_val).  Elements are at most GW_MAX_ELEMENT bytes long including the length word.
 * Synchronous; allocates its own scratch.  GW_E_INVALID on a corrupt stream ("Corrupt
 * stream, found tag"), GW_E_OUTPUT_FULL if rec_cap / wm_cap are too small. */
#define GW_MAX_ELEMENT 128
int  gw_decode_serialized(const void* d_bytes, int64_t nbytes, const gw_record_layout* layout,
                          int64_t* d_key, int64_t* d_ts, int64_t* d_value, int64_t rec_cap,
                          int64_t* d_wm_pos, int64_t* d_wm_val, int64_t wm_cap,
                          gw_decode_result* out, void* stream);
/* Decode and process one input channel's bytes on the operator: the records between
 * two watermarks go through gw_ingest, each watermark through gw_advance_watermark —
 * what StreamTaskNetworkInput.processElement does per element (RS/runtime/io/
 * AbstractStreamTaskNetworkInput.java:152-175, processElement :205-230) with a single
 * input channel's StatusWatermarkValve.  *consumed (may be NULL) as in
 * gw_decode_result; *rows_fired (may be NULL) counts the rows the watermarks fired.
 * One host synchronisation per call (the watermark positions): pass many buffers at
 * once. */
int  gw_ingest_serialized(gw_handle* h, const void* bytes, int64_t nbytes, const gw_record_layout* layout,
                          int64_t* consumed, int64_t* rows_fired);
/* Same, with the bytes in device memory, produced on `stream` (NULL = default stream). */
int  gw_ingest_serialized_device(gw_handle* h, const void* d_bytes, int64_t nbytes,
                                 const gw_record_layout* layout, void* stream, int64_t* consumed,
                                 int64_t* rows_fired);

/* Bounded input ended (BoundedOneInput.endInput) — equivalent to MAX_WATERMARK. */
int  gw_end_input(gw_handle* h, int64_t* rows_fired);

/* ---- output ---------------------------------------------------------------- */
int  gw_pending_rows(gw_handle* h, int64_t* n);
/* Copy up to cap pending rows (key, window start, window end, result) to host
 * arrays and remove them.  Returns GW_E_OUTPUT_FULL if rows remain. */
/* GW_FLAG_FIRST_ELEMENT handles: the batch with each record's payload (SumAggregator /
 * ComparableAggregator keep the first element's other fields, RS/api/functions/aggregation/
 * SumAggregator.java:66-76, ComparableAggregator.java:83-104), and rows with the payload of
 * their window's first element.  gw_ingest / gw_ingest_device return GW_E_INVALID on such
 * handles; gw_drain drains the rows without the payload. */
int  gw_ingest_payload(gw_handle* h, int64_t n, const int64_t* key, const int32_t* key_hash, const int64_t* ts,
                       const void* value, const int64_t* payload);
int  gw_ingest_payload_device(gw_handle* h, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                              const int64_t* d_ts, const void* d_value, const int64_t* d_payload, void* stream);
int  gw_drain_payload(gw_handle* h, int64_t* key, int64_t* start, int64_t* end, void* result, int64_t* payload,
                      int64_t cap, int64_t* n);
int  gw_drain(gw_handle* h, int64_t* key, int64_t* start, int64_t* end, void* result,
              int64_t cap, int64_t* n);
/* Zero-copy device view of the pending rows (for a device-side consumer). */
int  gw_rows_device(gw_handle* h, const int64_t** d_key, const int64_t** d_start,
                    const int64_t** d_end, const void** d_result, int64_t* n);
/* Drop all pending rows (after a device consumer read them). */
int  gw_clear_rows(gw_handle* h);

int64_t gw_late_dropped(const gw_handle* h);
/* Late-data side output (GW_FLAG_LATE_SIDE_OUTPUT; WindowedStream.sideOutputLateData, RS/api/
 * datastream/WindowedStream.java): the records WindowOperator.processElement skips as late
 * (isSkippedElement && isElementLate, WindowOperator.java:440-446) are kept, as the element
 * itself (key, timestamp, value bits), instead of being counted in numLateRecordsDropped, and
 * handed out here (sideOutput :587-588).  A record is pending from the ingest call that saw
 * it; gw_drain_late copies up to cap records and removes them (GW_E_OUTPUT_FULL if more
 * remain).  Without the flag both report 0 records. */
int  gw_pending_late(gw_handle* h, int64_t* n);
int  gw_drain_late(gw_handle* h, int64_t* key, int64_t* ts, void* value, int64_t cap, int64_t* n);
int  gw_get_stats(const gw_handle* h, gw_stats* out);
int  gw_synchronize(gw_handle* h);
/* hipStream_t the handle launches on (for ordering / event timing by callers). */
void* gw_stream(gw_handle* h);
/* Average device duration (ms) per launch of each kernel family since the last call,
 * measured with HIP events on the handle's stream.  which: 0 = ingest (per batch;
 * region path: pass 1), 1 = fire, 2 = region pass 2 + apply (per buffer flush).
 * which = 3: *launches = the fires enqueued right behind their flush, without a host
 * round trip between them (gw_advance_watermark's common case), *ms = 0. */
int  gw_kernel_time_ms(gw_handle* h, int which, double* ms, int64_t* launches);
/* enable: 0 off, 1 every launch, k > 1: the region path's pass 1 (one launch per batch, all
 * alike) is timed on every k-th batch only (two event records per timed launch cost host
 * time between batches); `launches` then counts the timed ones. */
int  gw_enable_kernel_timing(gw_handle* h, int enable);

/* ---- window stagger (stateless) ------------------------------------------ */
/* WindowStagger (RS/api/windowing/assigners/WindowStagger.java:27-60) applied to a tumbling
 * assigner's global offset as TumblingEventTimeWindows.assignWindows does at the first
 * element (TumblingEventTimeWindows.java:72-79): *offset_out = (global_offset + stagger) % size
 * (Java remainder), the offset to create the operator with.  stagger = 0 (ALIGNED),
 * (long)(random01 * size) (RANDOM: random01 is the caller's ThreadLocalRandom.nextDouble()),
 * or max(0, processing_time - TimeWindow.getWindowStartWithOffset(processing_time, 0, size))
 * (NATURAL).  GW_E_INVALID for size <= 0, |global_offset| >= size or random01 outside [0, 1). */
#define GW_STAGGER_ALIGNED 0
#define GW_STAGGER_RANDOM  1
#define GW_STAGGER_NATURAL 2
int  gw_window_stagger_offset(int32_t stagger, int64_t processing_time, double random01, int64_t size,
                              int64_t global_offset, int64_t* offset_out);

/* ---- key groups (stateless) ---------------------------------------------- */
int32_t gw_java_long_hash(int64_t key);             /* Long.hashCode                     */
int32_t gw_murmur_hash(int32_t code);               /* MathUtils.murmurHash              */
int32_t gw_key_group_for_hash(int32_t key_hash, int32_t max_parallelism);
int32_t gw_operator_for_key_group(int32_t max_parallelism, int32_t parallelism, int32_t kg);
int32_t gw_default_max_parallelism(int32_t parallelism);
/* Device kernel: kg[i] / owner[i] (either may be NULL) for n keys. */
int  gw_key_groups_device(int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                          int32_t max_parallelism, int32_t parallelism,
                          int32_t* d_kg, int32_t* d_owner, void* stream);
/* Device kernel: stable partition of (key, ts, value) by owner subtask
 * (KeyGroupStreamPartitioner).  Output columns are grouped by destination; counts[p]
 * (device int64[parallelism]) receives the number of records for subtask p.
 * d_scratch must hold gw_partition_scratch_bytes(n, parallelism) bytes. */
int64_t gw_partition_scratch_bytes(int64_t n, int32_t parallelism);
int  gw_partition_device(int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                         const int64_t* d_ts, const void* d_value,
                         int32_t max_parallelism, int32_t parallelism,
                         int64_t* d_key_out, int64_t* d_ts_out, void* d_value_out,
                         int64_t* d_counts, void* d_scratch, void* stream);

/* Packed exchange records -- this path's serialized form of the records RecordWriter.emit
 * ships to the key group's owner (flink-runtime/.../io/network/api/writer/RecordWriter.java:
 * 104-110, KeyGroupStreamPartitioner.java:55-64), chosen for xGMI: one 8-byte word per record
 * instead of 24 B of key, ts and value
 *   lo32 = key, hi32 = value << 4 | d        (d = pane - base_pane, 0 <= d < 16)
 * for records whose key is in [0, 2^32), whose value (if the batch has values) is in
 * [-2^27, 2^27), and whose pane floor((ts - offset) / pane) lies in [base_pane, base_pane + 16);
 * the others travel as (key, ts, value).  Unpacked, a record's timestamp is its pane's start,
 * which changes no window decision of a tumbling / sliding assigner with size >= slide and
 * pane = gcd(size, slide) (assignWindows, isWindowLate and the cleanup time depend on the pane
 * alone).  Not for sessions, size < slide, the late side output, first-element / minBy
 * handles or floating values: those need the record's own timestamp or value.
 * gw_pack_geom_init: pane = gcd(size, slide) and base_pane = the pane of `watermark` (the
 * operator's watermark before the batch: records of earlier panes travel unpacked);
 * GW_E_UNSUPPORTED when size < slide or watermark = Long.MIN_VALUE.
 * gw_pack_records / gw_unpack_records: the same packing on the host (fits[i] = 0: record i
 * does not pack). */
typedef struct gw_pack_geom {
    int64_t pane;
    int64_t offset;
    int64_t base_pane;
    int32_t enabled;
    int32_t pad;
} gw_pack_geom;
int  gw_pack_geom_init(gw_pack_geom* g, int64_t size, int64_t slide, int64_t offset, int64_t watermark);
int  gw_pack_records(int64_t n, const int64_t* key, const int64_t* ts, const int64_t* value, const gw_pack_geom* g,
                     uint64_t* words, uint8_t* fits);
int  gw_unpack_records(int64_t n, const uint64_t* words, const gw_pack_geom* g, int64_t* key, int64_t* ts,
                       int64_t* value);
/* Device: stable partition by owner with packing (g->enabled): counts[2q] packed words of
 * subtask q (in d_packed_out), counts[2q + 1] its other records (in the columns), buckets laid
 * out q-major (q's packed words, then its other records, then q + 1's ...) at positions of one
 * numbering into both outputs.  parallelism <= 128.  d_scratch: gw_partition_scratch_bytes(n,
 * 2 * parallelism).  gw_unpack_device: n words back to columns. */
int  gw_partition_packed_device(int64_t n, const int64_t* d_key, const int64_t* d_ts, const int64_t* d_value,
                                int32_t max_parallelism, int32_t parallelism, const gw_pack_geom* g,
                                uint64_t* d_packed_out, int64_t* d_key_out, int64_t* d_ts_out, int64_t* d_value_out,
                                int64_t* d_counts, void* d_scratch, void* stream);
/* The exchange's single-pass partition (ranks <= 16): owner q's records go to region q of
 * capacity cap >= n -- its packed words (g enabled, else none) at d_packed_out + q * cap, its
 * other records at d_key_out / d_ts_out / d_value_out + q * cap, both in arrival order; d_counts
 * as gw_partition_packed_device's ([2p] with g enabled, else [p]).  No histogram pass: a
 * region per owner lets each tile's positions follow from earlier tiles' counts alone.  g may
 * be NULL (no packing); scratch: gw_partition_scratch_bytes(n, 2p). */
int  gw_partition_regions_device(int64_t n, const int64_t* d_key, const int64_t* d_ts, const int64_t* d_value,
                                 int32_t max_parallelism, int32_t parallelism, const gw_pack_geom* g, int64_t cap,
                                 uint64_t* d_packed_out, int64_t* d_key_out, int64_t* d_ts_out,
                                 int64_t* d_value_out, int64_t* d_counts, void* d_scratch, void* stream);
int  gw_unpack_device(int64_t n, const uint64_t* d_words, const gw_pack_geom* g, int64_t* d_key, int64_t* d_ts,
                      int64_t* d_value, void* stream);
/* The stages a job chains ahead of keyBy on simple records, fused on the device (no Flink-core
 * interface: the Yahoo Streaming Benchmark's FilterFunction(event_type == view) + projection +
 * join against a static ad -> campaign table, AdvertisingTopologyNative): of the n records
 * whose d_sel[i] == sel_value, in arrival order, d_key_out[j] = d_dict[d_idx[i]] and
 * d_ts_out[j] = d_ts[i]; *n_out = their number (the call waits for it on `stream`).  An index
 * outside [0, dict_n) is GW_E_RANGE.  Outputs hold n records at most. */
int  gw_select_lookup_device(int64_t n, const int64_t* d_sel, int64_t sel_value, const int64_t* d_idx,
                             const int64_t* d_dict, int64_t dict_n, const int64_t* d_ts, int64_t* d_key_out,
                             int64_t* d_ts_out, int64_t* n_out, void* stream);
/* gw_ingest_device for a batch of n_other column records followed by n_words packed words
 * (the receive side of the packed exchange: what StreamTaskNetworkInput deserializes before
 * WindowOperator.processElement, WindowOperator.java:293-447, sees record by record)
 * (gw_exchange_last_words): the words' timestamps are their panes' starts (gw_pack_geom).  A
 * plain pane operator's region pass 1 decodes the words itself; the direct / pre-aggregation
 * paths and window-class handles get them unpacked first.  GW_E_UNSUPPORTED when n_words > 0
 * and the handle needs a record's own timestamp or value (sessions, count windows,
 * first-element / minBy handles, the late side output, floating aggregates) or when g's pane
 * does not divide the handle's size, slide and offset difference.  Column pointers may be NULL
 * when n_other = 0. */
int  gw_ingest_packed_device(gw_handle* h, int64_t n_other, const int64_t* d_key, const int64_t* d_ts,
                             const int64_t* d_value, int64_t n_words, const uint64_t* d_words,
                             const gw_pack_geom* g, void* stream);

/* ---- keyBy exchange over RCCL (one process per GPU) ------------------------
 * Replaces the network shuffle behind KeyGroupStreamPartitioner.selectChannel
 * (flink-runtime/.../streaming/runtime/partitioner/KeyGroupStreamPartitioner.java:55-64)
 * and RecordWriter.emit (flink-runtime/.../io/network/api/writer/RecordWriter.java:
 * 104-110): per watermark batch, the device partition above, an RCCL all-to-all of the
 * per-destination counts, then one grouped ncclSend/ncclRecv per column and peer over
 * xGMI.  The watermark combine of StatusWatermarkValve.inputWatermark (minimum over the
 * input channels, flink-streaming-java/.../watermarkstatus/StatusWatermarkValve.java:
 * 153-185) is an RCCL all-reduce(MIN).
 *
 * gw_exchange_unique_id: rank 0 creates the 128-byte communicator id; the caller hands it
 * to every rank out of band (the JobManager / a TCP rendezvous), each rank calls
 * gw_exchange_create with it.
 *
 * gw_exchange_batch: d_key/d_ts (d_value, d_key_hash may be NULL) hold this rank's n records
 * of one watermark batch and wm the watermark its source emitted after them.  One RCCL
 * all-to-all carries, per peer, (record count, watermark, column presence); the host waits
 * for it once (one device->host copy: the only host synchronisation of the batch), checks
 * that every rank sends the same columns (GW_E_INVALID otherwise, on every rank), then
 * enqueues one grouped ncclSend/ncclRecv per column and peer on `stream`.  Out: the *n_out
 * records this rank owns in receive columns owned by the exchange (*d_*_out; NULL for an
 * absent column), valid until GW_EXCHANGE_RECV_SETS batches later (receive sets used in turn);
 * *wm_out = the minimum of the ranks' watermarks (StatusWatermarkValve); *ingest_stream = a
 * hand-off stream of this receive set, ordered after the receives: pass it as the producer
 * stream of gw_ingest_device, whose "producer waits for my reads" ordering then lands on
 * the hand-off stream, so the exchange of the next batch never waits for this batch's
 * ingest, only the reuse of this receive set GW_EXCHANGE_RECV_SETS batches later does; that
 * ordering is taken when the later batch is finished, so a driver that finishes batches ahead of
 * the ingest (e.g. from a thread of its own) finishes batch b only once the ingest of batch
 * b - GW_EXCHANGE_RECV_SETS has been issued.  All ranks call it
 * for every batch (n may be 0).  gw_exchange_counts: the last batch's per-peer send and
 * receive record counts (nranks each; either may be NULL).
 *
 * Failure: no host wait of the exchange is unbounded (a failed channel fails the task in the
 * reference; here a dead or diverging peer would otherwise leave every rank spinning in RCCL).
 * Each wait polls the stream, ncclCommGetAsyncError and a deadline (gw_exchange_set_timeout,
 * default 60000 ms; 0: none); on a stream error, an asynchronous RCCL error or expiry the
 * communicator is aborted (ncclCommAbort) and the call returns GW_E_STATE with the reason in
 * gw_exchange_last_error.  Every later call on that exchange returns GW_E_STATE; destroy it
 * and fail the task (the JVM side throws, GpuKeyByExchange.java). */
#define GW_EXCHANGE_ID_BYTES 128
#define GW_EXCHANGE_RECV_SETS 3
typedef struct gw_exchange gw_exchange;
int  gw_exchange_unique_id(void* id);
int  gw_exchange_create(gw_exchange** out, int32_t nranks, int32_t rank, const void* id, int32_t device,
                        int32_t max_parallelism);
void gw_exchange_destroy(gw_exchange* ex);
int  gw_exchange_set_timeout(gw_exchange* ex, int64_t timeout_ms);
/* gw_exchange_batch in two halves, so no host wait sits between batches: gw_exchange_begin
 * partitions a batch and queues its count all-to-all (no wait); gw_exchange_finish takes the
 * oldest begun batch, waits for its counts (the batch's one host wait, bounded as above),
 * queues the sends / receives and returns what gw_exchange_batch returns.  Up to two batches
 * may be begun and not finished (GW_E_STATE beyond); issue begin(b + 1) before finish(b) and
 * the partition of b + 1 runs while the host waits for b's counts.  Both halves of a batch
 * on the same stream.  Each call selects the exchange's device for the calling thread, so the
 * exchange may run on a host thread of its own (one thread per exchange at a time).  Packing takes its base pane from the combined watermark of the last
 * batch finished before the begin (the same on every rank, which begin and finish in the
 * same order). */
int  gw_exchange_begin(gw_exchange* ex, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                       const int64_t* d_ts, const int64_t* d_value, int64_t wm, void* stream);
int  gw_exchange_finish(gw_exchange* ex, int64_t* n_out, const int64_t** d_key_out, const int32_t** d_key_hash_out,
                        const int64_t** d_ts_out, const int64_t** d_value_out, int64_t* wm_out, void** ingest_stream,
                        void* stream);
int  gw_exchange_batch(gw_exchange* ex, int64_t n, const int64_t* d_key, const int32_t* d_key_hash,
                       const int64_t* d_ts, const int64_t* d_value, int64_t wm, int64_t* n_out,
                       const int64_t** d_key_out, const int32_t** d_key_hash_out, const int64_t** d_ts_out,
                       const int64_t** d_value_out, int64_t* wm_out, void** ingest_stream, void* stream);
int  gw_exchange_counts(const gw_exchange* ex, int64_t* send, int64_t* recv);
/* Packing (gw_pack_geom above) for the following batches of a tumbling / sliding operator
 * (size >= slide) without the late side output: from the second batch on, the records that
 * fit travel as 8-byte words (base pane: the previous batch's combined watermark) and arrive
 * unpacked, behind the records that did not fit; per key the arrival order then differs, so
 * only for integer aggregates (with_values: the value column is an integer sum / min / max /
 * count operand).  Every rank must enable it alike (else GW_E_INVALID on every rank at the
 * next batch).  gw_exchange_last_packed: records this rank received packed in the last batch. */
int  gw_exchange_enable_packing(gw_exchange* ex, int64_t size, int64_t slide, int64_t offset, int32_t with_values);
int64_t gw_exchange_last_packed(const gw_exchange* ex);
/* gw_exchange_set_unpack(ex, 0): the received words stay packed -- gw_exchange_batch's
 * *n_out and columns then hold only the records that travelled unpacked, and
 * gw_exchange_last_words gives the words (device, valid like the columns) and their geometry
 * for gw_ingest_packed_device, whose region pass 1 decodes them (8 B read per record instead
 * of an unpack pass writing 24 B that pass 1 reads again). */
int  gw_exchange_set_unpack(gw_exchange* ex, int32_t unpack);
int  gw_exchange_last_words(const gw_exchange* ex, int64_t* n_words, const uint64_t** d_words, gw_pack_geom* g);
int  gw_exchange_min_watermark(gw_exchange* ex, int64_t wm, int64_t* out, void* stream);
const char* gw_exchange_last_error(const gw_exchange* ex);
/* The per-peer plan gw_exchange_batch runs after its count all-to-all, as a host function
 * (no device, no communicator): from the messages this rank sent and received --
 * msg[4q .. 4q+3] = (records, watermark, column mask, packed records) for peer q -- the
 * offsets and counts of every send and receive (send_off[q]: the first record for q in the
 * rank's owner-partitioned numbering; recv_off[q]: where q's records land when nothing is
 * packed: the receive columns hold the peers' records in rank order, as all_to_all_single
 * lays them out), the total received and the minimum watermark over the ranks
 * (StatusWatermarkValve).  GW_E_INVALID when a peer's column mask (value column, key hashes,
 * packing) differs from this rank's.
 * gw_exchange_plan_packed: the packed split -- send_packed[q] of q's records are words (at
 * send_off[q]), the rest follow them; q's unpacked-in-transit records land at
 * recv_other_off[q] of the receive columns, its words at recv_packed_off[q] of the word
 * buffer (recv_packed[q] of them), and are unpacked to positions total_other + recv_packed_off[q]. */
int  gw_exchange_plan(int32_t nranks, const int64_t* sent_msg, const int64_t* recv_msg, int64_t cols_mask,
                      int64_t wm, int64_t* send_off, int64_t* send_cnt, int64_t* recv_off, int64_t* recv_cnt,
                      int64_t* total, int64_t* wm_min);
int  gw_exchange_plan_packed(int32_t nranks, const int64_t* sent_msg, const int64_t* recv_msg, int64_t* send_packed,
                             int64_t* recv_other_off, int64_t* recv_packed_off, int64_t* recv_packed,
                             int64_t* total_other, int64_t* total_packed);

#ifdef __cplusplus
}
#endif
#endif /* GPUWIN_H */
