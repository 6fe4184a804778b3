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
                                          jlong capacityHint, jlong maxBatch) {
    gw_config cfg = {assigner, trigger, size, slide, offset, gap, lateness, agg, maxParallelism,
                     parallelism, subtask, device, 0, capacityHint, maxBatch};
    gw_handle* h = 0;
    int rc = gw_create(&cfg, &h);
    if (rc) { fail(env, 0, rc); return 0; }
    return (jlong)(intptr_t)h;
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

JNIEXPORT jlong JNICALL CLS(nativeLateDropped)(JNIEnv* env, jclass c, jlong h) {
    return gw_late_dropped((gw_handle*)(intptr_t)h);
}

JNIEXPORT void JNICALL CLS(nativeDestroy)(JNIEnv* env, jclass c, jlong h) { gw_destroy((gw_handle*)(intptr_t)h); }
