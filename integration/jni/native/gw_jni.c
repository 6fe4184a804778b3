/*
 * gw_jni.c — JNI glue between GpuWindowOperator.java and libgpuwin.so (include/gpuwin.h).
 * NOT BUILT in this repository (no JDK in the build image); a Flink maintainer compiles it
 * with:  gcc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I<repo>/include \
 *            gw_jni.c -L<repo>/flink_amd -lgpuwin -o libgpuwin_jni.so
 * Columns travel as direct ByteBuffers (off-heap, no copy at the JNI boundary); a negative
 * status becomes a java.lang.RuntimeException carrying gw_last_error(), which fails the
 * task exactly like an exception thrown by WindowOperator.processElement/onEventTime.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "gpuwin.h"

#define CLS(n) Java_org_apache_flink_streaming_runtime_operators_windowing_gpu_GpuWindowOperator_##n

static jint fail(JNIEnv* env, gw_handle* h, int rc) {
    if (rc < 0 && rc != GW_E_OUTPUT_FULL) {
        jclass ex = (*env)->FindClass(env, rc == GW_E_INVALID ? "java/lang/IllegalArgumentException"
                                                             : "java/lang/RuntimeException");
        (*env)->ThrowNew(env, ex, gw_last_error(h));
    }
    return rc;
}

JNIEXPORT jlong JNICALL CLS(nativeCreate)(JNIEnv* env, jclass c, jint assigner, jint trigger, jlong size,
                                          jlong slide, jlong offset, jlong gap, jlong lateness, jint agg,
                                          jint maxParallelism, jint parallelism, jint subtask, jint device,
                                          jint flags, jlong capacityHint, jlong maxBatch) {
    gw_config cfg = {assigner, trigger, size, slide, offset, gap, lateness, agg, maxParallelism,
                     parallelism, subtask, device, flags, capacityHint, maxBatch};
    gw_handle* h = 0;
    int rc = gw_create(&cfg, &h);
    if (rc) { fail(env, 0, rc); return 0; }
    return (jlong)(intptr_t)h;
}

/* TumblingEventTimeWindows' stagger at the first element: the offset GpuWindowOperator
 * creates its handle with (gw_window_stagger_offset). */
JNIEXPORT jlong JNICALL CLS(nativeStaggerOffset)(JNIEnv* env, jclass c, jint stagger, jlong processingTime,
                                                 jdouble random01, jlong size, jlong globalOffset) {
    int64_t off = 0;
    int rc = gw_window_stagger_offset(stagger, processingTime, random01, size, globalOffset, &off);
    if (rc) fail(env, 0, rc);
    return off;
}

/* keys/ts/values/keyHashes: direct ByteBuffers of n little-endian longs / ints */
JNIEXPORT void JNICALL CLS(nativeIngest)(JNIEnv* env, jclass c, jlong h, jint n, jobject keys, jobject keyHashes,
                                         jobject ts, jobject values) {
    const int64_t* k = (*env)->GetDirectBufferAddress(env, keys);
    const int32_t* kh = keyHashes ? (*env)->GetDirectBufferAddress(env, keyHashes) : 0;
    const int64_t* t = (*env)->GetDirectBufferAddress(env, ts);
    const void* v = values ? (*env)->GetDirectBufferAddress(env, values) : 0;
    fail(env, (gw_handle*)(intptr_t)h, gw_ingest((gw_handle*)(intptr_t)h, n, k, kh, t, v));
}

/* Staged ingest (gw_stage_*): the operator's column buffers are the library's pinned slots, so
 * processElement writes each record straight into the memory the PCIe transfer reads.
 * nativeStageAlloc returns the status without throwing: GW_E_UNSUPPORTED (a composite or
 * first-element handle) leaves the operator on its own direct buffers and nativeIngest. */
JNIEXPORT jint JNICALL CLS(nativeStageAlloc)(JNIEnv* env, jclass c, jlong h, jint slots, jint cap) {
    return gw_stage_alloc((gw_handle*)(intptr_t)h, slots, cap);
}

/* Column `which` (0 key, 1 key hash, 2 timestamp, 3 value) of a slot as a direct ByteBuffer of
 * cap entries, once the slot's previous transfer has read it. */
JNIEXPORT jobject JNICALL CLS(nativeStageColumn)(JNIEnv* env, jclass c, jlong h, jint slot, jint which, jint cap) {
    gw_handle* g = (gw_handle*)(intptr_t)h;
    int64_t *k = 0, *t = 0, *v = 0;
    int32_t* kh = 0;
    int rc = gw_stage_columns(g, slot, &k, &kh, &t, &v);
    if (rc) {
        fail(env, g, rc);
        return 0;
    }
    void* p = which == 0 ? (void*)k : which == 1 ? (void*)kh : which == 2 ? (void*)t : (void*)v;
    return (*env)->NewDirectByteBuffer(env, p, (jlong)cap * (which == 1 ? 4 : 8));
}

/* The slot's first n records (cols: GW_STAGE_VALUE | GW_STAGE_KEY_HASH). */
JNIEXPORT void JNICALL CLS(nativeIngestStage)(JNIEnv* env, jclass c, jlong h, jint slot, jint n, jint cols) {
    gw_handle* g = (gw_handle*)(intptr_t)h;
    fail(env, g, gw_ingest_stage(g, slot, n, cols));
}

/* A complete slot sent over PCIe ahead of its nativeIngestStage (gw_stage_send). */
JNIEXPORT void JNICALL CLS(nativeStageSend)(JNIEnv* env, jclass c, jlong h, jint slot, jint n, jint cols) {
    gw_handle* g = (gw_handle*)(intptr_t)h;
    fail(env, g, gw_stage_send(g, slot, n, cols));
}

/* Network-buffer ingest: `bytes` is a direct ByteBuffer holding one input channel's
 * serialized elements (the payload of its network buffers, in order); `types` the Tuple's
 * field type codes ("JJ" for Tuple2<Long, Long>).  Returns the bytes consumed; the caller
 * keeps the rest (an element spanning into the next buffer).  Rows fired by the channel's
 * watermarks are drained as usual. */
JNIEXPORT jlong JNICALL CLS(nativeIngestSerialized)(JNIEnv* env, jclass c, jlong h, jobject bytes, jlong n,
                                                    jstring types, jint keyField, jint valueField) {
    gw_record_layout lay;
    memset(&lay, 0, sizeof(lay));
    const char* t = (*env)->GetStringUTFChars(env, types, 0);
    lay.nfields = (int32_t)strlen(t);
    if (lay.nfields > GW_MAX_FIELDS) lay.nfields = GW_MAX_FIELDS + 1; /* rejected by gw_ingest_serialized */
    memcpy(lay.types, t, lay.nfields <= GW_MAX_FIELDS ? (size_t)lay.nfields : 0);
    (*env)->ReleaseStringUTFChars(env, types, t);
    lay.key_field = keyField;
    lay.value_field = valueField;
    int64_t consumed = 0, rows = 0;
    fail(env, (gw_handle*)(intptr_t)h,
         gw_ingest_serialized((gw_handle*)(intptr_t)h, (*env)->GetDirectBufferAddress(env, bytes), n, &lay,
                              &consumed, &rows));
    return consumed;
}

JNIEXPORT jlong JNICALL CLS(nativeAdvanceWatermark)(JNIEnv* env, jclass c, jlong h, jlong wm) {
    int64_t rows = 0;
    fail(env, (gw_handle*)(intptr_t)h, gw_advance_watermark((gw_handle*)(intptr_t)h, wm, &rows));
    return rows;
}

/* Drains up to cap rows into four direct buffers; returns the count (more may remain). */
JNIEXPORT jint JNICALL CLS(nativeDrain)(JNIEnv* env, jclass c, jlong h, jobject key, jobject start, jobject end,
                                        jobject result, jint cap) {
    int64_t n = 0;
    int rc = gw_drain((gw_handle*)(intptr_t)h, (*env)->GetDirectBufferAddress(env, key),
                      (*env)->GetDirectBufferAddress(env, start), (*env)->GetDirectBufferAddress(env, end),
                      (*env)->GetDirectBufferAddress(env, result), cap, &n);
    fail(env, (gw_handle*)(intptr_t)h, rc);
    return (jint)n;
}

/* Positional sum/min/max on Tuple3+ (GW_FLAG_FIRST_ELEMENT): the batch with a payload column
 * (the operator's arrival sequence of each element) ... */
JNIEXPORT void JNICALL CLS(nativeIngestPayload)(JNIEnv* env, jclass c, jlong h, jint n, jobject keys,
                                                jobject keyHashes, jobject ts, jobject values, jobject payload) {
    gw_handle* g = (gw_handle*)(intptr_t)h;
    fail(env, g, gw_ingest_payload(g, n, (*env)->GetDirectBufferAddress(env, keys),
                                   keyHashes ? (*env)->GetDirectBufferAddress(env, keyHashes) : 0,
                                   (*env)->GetDirectBufferAddress(env, ts), (*env)->GetDirectBufferAddress(env, values),
                                   (*env)->GetDirectBufferAddress(env, payload)));
}

/* ... and rows with their window's first-element payload: up to cap rows into five direct
 * buffers; returns the count (more may remain). */
JNIEXPORT jint JNICALL CLS(nativeDrainPayload)(JNIEnv* env, jclass c, jlong h, jobject key, jobject start,
                                               jobject end, jobject result, jobject payload, jint cap) {
    gw_handle* g = (gw_handle*)(intptr_t)h;
    int64_t n = 0;
    int rc = gw_drain_payload(g, (*env)->GetDirectBufferAddress(env, key), (*env)->GetDirectBufferAddress(env, start),
                              (*env)->GetDirectBufferAddress(env, end), (*env)->GetDirectBufferAddress(env, result),
                              (*env)->GetDirectBufferAddress(env, payload), cap, &n);
    fail(env, g, rc);
    return (jint)n;
}

JNIEXPORT jlong JNICALL CLS(nativeLateDropped)(JNIEnv* env, jclass c, jlong h) {
    return gw_late_dropped((gw_handle*)(intptr_t)h);
}

JNIEXPORT void JNICALL CLS(nativeDestroy)(JNIEnv* env, jclass c, jlong h) { gw_destroy((gw_handle*)(intptr_t)h); }

/* prepareSnapshotPreBarrier: apply every buffered record (gw_flush). */
JNIEXPORT void JNICALL CLS(nativeFlush)(JNIEnv* env, jclass c, jlong h) {
    fail(env, (gw_handle*)(intptr_t)h, gw_flush((gw_handle*)(intptr_t)h));
}

/* snapshotState: the window state of key groups [lo, hi] as one blob (gw_snapshot). */
JNIEXPORT jbyteArray JNICALL CLS(nativeSnapshot)(JNIEnv* env, jclass c, jlong h, jint lo, jint hi) {
    gw_handle* g = (gw_handle*)(intptr_t)h;
    int64_t len = 0;
    if (fail(env, g, gw_snapshot(g, lo, hi, 0, 0, &len)) < 0) return 0;
    void* buf = malloc((size_t)len);
    int rc = gw_snapshot(g, lo, hi, buf, len, &len);
    jbyteArray out = 0;
    if (rc == GW_OK) {
        out = (*env)->NewByteArray(env, (jsize)len);
        (*env)->SetByteArrayRegion(env, out, 0, (jsize)len, (const jbyte*)buf);
    }
    free(buf);
    fail(env, g, rc);
    return out;
}

/* The part of a [lo, hi] snapshot blob that belongs to key group kg, as a blob of its own
 * (written per key group into the raw keyed state stream).  gw_snapshot_slice reads the
 * entry size from the blob header, so pane, session and count-window blobs all slice. */
JNIEXPORT jbyteArray JNICALL CLS(nativeSliceKeyGroup)(JNIEnv* env, jclass c, jbyteArray blob, jint kg) {
    jsize len = (*env)->GetArrayLength(env, blob);
    jbyte* b = (*env)->GetByteArrayElements(env, blob, 0);
    int64_t out_len = 0;
    int rc = gw_snapshot_slice(b, len, kg, 0, 0, &out_len);
    jbyteArray out = 0;
    if (rc == GW_OK) {
        void* tmp = malloc((size_t)out_len);
        rc = tmp ? gw_snapshot_slice(b, len, kg, tmp, out_len, &out_len) : GW_E_OOM;
        if (rc == GW_OK) {
            out = (*env)->NewByteArray(env, (jsize)out_len);
            (*env)->SetByteArrayRegion(env, out, 0, (jsize)out_len, (const jbyte*)tmp);
        }
        free(tmp);
    }
    (*env)->ReleaseByteArrayElements(env, blob, b, JNI_ABORT);
    fail(env, 0, rc);
    return out;
}

/* initializeState: restore one key group's blob (gw_restore). */
JNIEXPORT void JNICALL CLS(nativeRestore)(JNIEnv* env, jclass c, jlong h, jbyteArray blob) {
    jsize len = (*env)->GetArrayLength(env, blob);
    jbyte* b = (*env)->GetByteArrayElements(env, blob, 0);
    int rc = gw_restore((gw_handle*)(intptr_t)h, b, len);
    (*env)->ReleaseByteArrayElements(env, blob, b, JNI_ABORT);
    fail(env, (gw_handle*)(intptr_t)h, rc);
}

/* Device-resident ingest (gw_ingest_device): the columns the keyBy exchange delivered
 * (GpuKeyByExchange.batch), as raw device addresses; 0 = absent column.  `stream` is the
 * stream that produced them (the exchange's): the handle's stream waits for it before
 * reading, and it waits for those reads before the exchange reuses the receive set. */
JNIEXPORT void JNICALL CLS(nativeIngestDevice)(JNIEnv* env, jclass c, jlong h, jlong n, jlong keyPtr, jlong hashPtr,
                                               jlong tsPtr, jlong valuePtr, jlong stream) {
    gw_handle* g = (gw_handle*)(intptr_t)h;
    fail(env, g, gw_ingest_device(g, n, (const int64_t*)(intptr_t)keyPtr, (const int32_t*)(intptr_t)hashPtr,
                                  (const int64_t*)(intptr_t)tsPtr, (const void*)(intptr_t)valuePtr,
                                  (void*)(intptr_t)stream));
}

/* The key ids a key group's blob names (gw_snapshot_keys): snapshotState writes the real key
 * of each through the key serializer after the blob. */
JNIEXPORT jlongArray JNICALL CLS(nativeSnapshotKeys)(JNIEnv* env, jclass c, jbyteArray blob) {
    jsize len = (*env)->GetArrayLength(env, blob);
    jbyte* b = (*env)->GetByteArrayElements(env, blob, 0);
    int64_t n = 0;
    int rc = gw_snapshot_keys(b, len, 0, 0, &n);
    jlongArray out = 0;
    if (rc == GW_OK) {
        int64_t* tmp = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
        rc = tmp ? gw_snapshot_keys(b, len, tmp, n, &n) : GW_E_OOM;
        if (rc == GW_OK) {
            out = (*env)->NewLongArray(env, (jsize)n);
            (*env)->SetLongArrayRegion(env, out, 0, (jsize)n, (const jlong*)tmp);
        }
        free(tmp);
    }
    (*env)->ReleaseByteArrayElements(env, blob, b, JNI_ABORT);
    fail(env, 0, rc);
    return out;
}

/* initializeState: the restored blob's key ids -> this subtask's ids (ascending `from`),
 * rewritten in place (gw_snapshot_remap_keys). */
JNIEXPORT void JNICALL CLS(nativeRemapKeys)(JNIEnv* env, jclass c, jbyteArray blob, jlongArray from, jlongArray to) {
    jsize len = (*env)->GetArrayLength(env, blob);
    jsize n = (*env)->GetArrayLength(env, from);
    jbyte* b = (*env)->GetByteArrayElements(env, blob, 0);
    jlong* f = (*env)->GetLongArrayElements(env, from, 0);
    jlong* t = (*env)->GetLongArrayElements(env, to, 0);
    int rc = (*env)->GetArrayLength(env, to) == n ? gw_snapshot_remap_keys(b, len, (const int64_t*)f, (const int64_t*)t, n)
                                                   : GW_E_INVALID;
    (*env)->ReleaseLongArrayElements(env, to, t, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, from, f, JNI_ABORT);
    (*env)->ReleaseByteArrayElements(env, blob, b, rc == GW_OK ? 0 : JNI_ABORT);  /* 0: copy back */
    fail(env, 0, rc);
}

/* sideOutputLateData: up to cap late records into direct buffers (key, timestamp, value);
 * returns how many were copied (more may remain: call again). */
JNIEXPORT jint JNICALL CLS(nativeDrainLate)(JNIEnv* env, jclass c, jlong h, jobject key, jobject ts, jobject value,
                                            jint cap) {
    gw_handle* g = (gw_handle*)(intptr_t)h;
    int64_t n = 0;
    int rc = gw_drain_late(g, (*env)->GetDirectBufferAddress(env, key), (*env)->GetDirectBufferAddress(env, ts),
                           value ? (*env)->GetDirectBufferAddress(env, value) : 0, cap, &n);
    fail(env, g, rc);
    return (jint)n;
}

/* First-element blobs: the payloads (ElementLog ids) their entries name, ascending, and in
 * maxEnd[0] the latest window end (gw_snapshot_payloads). */
JNIEXPORT jlongArray JNICALL CLS(nativeSnapshotPayloads)(JNIEnv* env, jclass c, jbyteArray blob, jlongArray maxEnd) {
    jsize len = (*env)->GetArrayLength(env, blob);
    jbyte* b = (*env)->GetByteArrayElements(env, blob, 0);
    int64_t n = 0, mx = 0;
    int rc = gw_snapshot_payloads(b, len, 0, 0, &n, &mx);
    jlongArray out = 0;
    if (rc == GW_OK) {
        int64_t* tmp = (int64_t*)malloc((size_t)(n > 0 ? n : 1) * 8);
        rc = tmp ? gw_snapshot_payloads(b, len, tmp, n, &n, &mx) : GW_E_OOM;
        if (rc == GW_OK) {
            out = (*env)->NewLongArray(env, (jsize)n);
            (*env)->SetLongArrayRegion(env, out, 0, (jsize)n, (const jlong*)tmp);
            (*env)->SetLongArrayRegion(env, maxEnd, 0, 1, (const jlong*)&mx);
        }
        free(tmp);
    }
    (*env)->ReleaseByteArrayElements(env, blob, b, JNI_ABORT);
    fail(env, 0, rc);
    return out;
}

/* ... and rewritten to this subtask's ElementLog ids (ascending `from`), in place. */
JNIEXPORT void JNICALL CLS(nativeRemapPayloads)(JNIEnv* env, jclass c, jbyteArray blob, jlongArray from,
                                                jlongArray to) {
    jsize len = (*env)->GetArrayLength(env, blob);
    jsize n = (*env)->GetArrayLength(env, from);
    jbyte* b = (*env)->GetByteArrayElements(env, blob, 0);
    jlong* f = (*env)->GetLongArrayElements(env, from, 0);
    jlong* t = (*env)->GetLongArrayElements(env, to, 0);
    int rc = (*env)->GetArrayLength(env, to) == n
                 ? gw_snapshot_remap_payloads(b, len, (const int64_t*)f, (const int64_t*)t, n)
                 : GW_E_INVALID;
    (*env)->ReleaseLongArrayElements(env, to, t, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, from, f, JNI_ABORT);
    (*env)->ReleaseByteArrayElements(env, blob, b, rc == GW_OK ? 0 : JNI_ABORT);
    fail(env, 0, rc);
}

/* ---- GpuKeyByExchange: the keyBy shuffle through libgpuwin's RCCL communicator ---- */
#define XCLS(n) Java_org_apache_flink_streaming_runtime_operators_windowing_gpu_GpuKeyByExchange_##n

static jint fail_ex(JNIEnv* env, gw_exchange* x, int rc) {
    if (rc < 0) {
        /* GW_E_STATE: the communicator was aborted (a peer died or diverged, an asynchronous
         * RCCL error, a wait past gw_exchange_set_timeout): the task fails */
        jclass ex = (*env)->FindClass(env, rc == GW_E_INVALID ? "java/lang/IllegalArgumentException"
                                           : rc == GW_E_STATE ? "java/lang/IllegalStateException"
                                                              : "java/lang/RuntimeException");
        (*env)->ThrowNew(env, ex, x ? gw_exchange_last_error(x) : "gw_exchange: invalid argument or device error");
    }
    return rc;
}

/* Rank 0: the communicator id into a direct buffer of GW_EXCHANGE_ID_BYTES bytes (shipped to
 * the other subtasks through the job's own channel). */
JNIEXPORT void JNICALL XCLS(nativeUniqueId)(JNIEnv* env, jclass c, jobject id) {
    fail_ex(env, 0, gw_exchange_unique_id((*env)->GetDirectBufferAddress(env, id)));
}

JNIEXPORT jlong JNICALL XCLS(nativeCreate)(JNIEnv* env, jclass c, jint nranks, jint rank, jobject id, jint device,
                                           jint maxParallelism) {
    gw_exchange* x = 0;
    int rc = gw_exchange_create(&x, nranks, rank, (*env)->GetDirectBufferAddress(env, id), device, maxParallelism);
    if (rc) { fail_ex(env, 0, rc); return 0; }
    return (jlong)(intptr_t)x;
}

JNIEXPORT void JNICALL XCLS(nativeDestroy)(JNIEnv* env, jclass c, jlong x) {
    gw_exchange_destroy((gw_exchange*)(intptr_t)x);
}

/* One watermark batch: device columns in (raw addresses, 0 = absent) and the watermark the
 * source emitted after them; `out` is a direct buffer of 7 longs receiving {records received,
 * key, key hash, timestamp, value device addresses, minimum watermark over the subtasks, the
 * ingest stream to pass to nativeIngestDevice}. */
JNIEXPORT void JNICALL XCLS(nativeBatch)(JNIEnv* env, jclass c, jlong x, jlong n, jlong keyPtr, jlong hashPtr,
                                         jlong tsPtr, jlong valuePtr, jlong wm, jlong stream, jobject out) {
    int64_t* o = (*env)->GetDirectBufferAddress(env, out);
    const int64_t *k = 0, *t = 0, *v = 0;
    const int32_t* kh = 0;
    void* ist = 0;
    int rc = gw_exchange_batch((gw_exchange*)(intptr_t)x, n, (const int64_t*)(intptr_t)keyPtr,
                               (const int32_t*)(intptr_t)hashPtr, (const int64_t*)(intptr_t)tsPtr,
                               (const int64_t*)(intptr_t)valuePtr, wm, &o[0], &k, &kh, &t, &v, &o[5], &ist,
                               (void*)(intptr_t)stream);
    o[1] = (int64_t)(intptr_t)k;
    o[2] = (int64_t)(intptr_t)kh;
    o[3] = (int64_t)(intptr_t)t;
    o[4] = (int64_t)(intptr_t)v;
    o[6] = (int64_t)(intptr_t)ist;
    fail_ex(env, (gw_exchange*)(intptr_t)x, rc);
}

/* The same batch in two halves, one batch ahead (gw_exchange_begin / gw_exchange_finish): begin
 * partitions and queues the count all-to-all without a host wait; finish fills `out` as
 * nativeBatch does for the oldest begun batch. */
JNIEXPORT void JNICALL XCLS(nativeBegin)(JNIEnv* env, jclass c, jlong x, jlong n, jlong keyPtr, jlong hashPtr,
                                         jlong tsPtr, jlong valuePtr, jlong wm, jlong stream) {
    fail_ex(env, (gw_exchange*)(intptr_t)x,
            gw_exchange_begin((gw_exchange*)(intptr_t)x, n, (const int64_t*)(intptr_t)keyPtr,
                              (const int32_t*)(intptr_t)hashPtr, (const int64_t*)(intptr_t)tsPtr,
                              (const int64_t*)(intptr_t)valuePtr, wm, (void*)(intptr_t)stream));
}

JNIEXPORT void JNICALL XCLS(nativeFinish)(JNIEnv* env, jclass c, jlong x, jlong stream, jobject out) {
    int64_t* o = (*env)->GetDirectBufferAddress(env, out);
    const int64_t *k = 0, *t = 0, *v = 0;
    const int32_t* kh = 0;
    void* ist = 0;
    int rc = gw_exchange_finish((gw_exchange*)(intptr_t)x, &o[0], &k, &kh, &t, &v, &o[5], &ist,
                                (void*)(intptr_t)stream);
    o[1] = (int64_t)(intptr_t)k;
    o[2] = (int64_t)(intptr_t)kh;
    o[3] = (int64_t)(intptr_t)t;
    o[4] = (int64_t)(intptr_t)v;
    o[6] = (int64_t)(intptr_t)ist;
    fail_ex(env, (gw_exchange*)(intptr_t)x, rc);
}

/* Packed records from the next batch on (gw_exchange_enable_packing): a tumbling / sliding
 * operator with size >= slide, no late side output, integer aggregate. */
JNIEXPORT void JNICALL XCLS(nativeEnablePacking)(JNIEnv* env, jclass c, jlong x, jlong size, jlong slide,
                                                 jlong offset, jboolean withValues) {
    fail_ex(env, (gw_exchange*)(intptr_t)x,
            gw_exchange_enable_packing((gw_exchange*)(intptr_t)x, size, slide, offset, withValues ? 1 : 0));
}

JNIEXPORT void JNICALL XCLS(nativeSetTimeout)(JNIEnv* env, jclass c, jlong x, jlong timeoutMs) {
    fail_ex(env, (gw_exchange*)(intptr_t)x, gw_exchange_set_timeout((gw_exchange*)(intptr_t)x, timeoutMs));
}

/* StatusWatermarkValve: the minimum of the subtasks' watermarks. */
JNIEXPORT jlong JNICALL XCLS(nativeMinWatermark)(JNIEnv* env, jclass c, jlong x, jlong wm, jlong stream) {
    int64_t out = wm;
    fail_ex(env, (gw_exchange*)(intptr_t)x,
            gw_exchange_min_watermark((gw_exchange*)(intptr_t)x, wm, &out, (void*)(intptr_t)stream));
    return out;
}
