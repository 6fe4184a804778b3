/* TEST-ONLY: a JNIEnv implementation (tests/jni/jni.h) so tests/test_jni_glue.py can call the
 * JNI glue of integration/jni/native/gw_jni.c from Python.  Byte arrays and strings are plain
 * C objects; direct ByteBuffers are passed as the raw address; ThrowNew records the pending
 * exception. */
#include <stdlib.h>
#include <string.h>
#include "jni.h"

typedef struct { jsize len; jbyte data[]; } fake_bytes;
static char g_exc_class[256], g_exc_msg[1024];
static int g_exc;

static jclass f_find_class(JNIEnv* e, const char* n) { (void)e; return (jclass)strdup(n); }
static jint f_throw_new(JNIEnv* e, jclass c, const char* m) {
    (void)e;
    g_exc = 1;
    strncpy(g_exc_class, (const char*)c, sizeof g_exc_class - 1);
    strncpy(g_exc_msg, m ? m : "", sizeof g_exc_msg - 1);
    free(c);
    return 0;
}
static void* f_direct(JNIEnv* e, jobject b) { (void)e; return (void*)b; }
static const char* f_utf(JNIEnv* e, jstring s, jboolean* c) { (void)e; if (c) *c = 0; return (const char*)s; }
static void f_rel_utf(JNIEnv* e, jstring s, const char* c) { (void)e; (void)s; (void)c; }
static jsize f_len(JNIEnv* e, jarray a) { (void)e; return ((fake_bytes*)a)->len; }
static jbyte* f_bytes(JNIEnv* e, jbyteArray a, jboolean* c) { (void)e; if (c) *c = 0; return ((fake_bytes*)a)->data; }
static void f_rel_bytes(JNIEnv* e, jbyteArray a, jbyte* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jbyteArray f_new_bytes(JNIEnv* e, jsize n) {
    (void)e;
    fake_bytes* b = (fake_bytes*)calloc(1, sizeof(fake_bytes) + (size_t)n);
    b->len = n;
    return (jbyteArray)b;
}
static void f_set_region(JNIEnv* e, jbyteArray a, jsize s, jsize n, const jbyte* src) {
    (void)e;
    memcpy(((fake_bytes*)a)->data + s, src, (size_t)n);
}

/* long[]: the same length-first layout, so GetArrayLength serves both */
typedef struct { jsize len; jlong data[]; } fake_longs;
static jlong* f_longs(JNIEnv* e, jlongArray a, jboolean* c) { (void)e; if (c) *c = 0; return ((fake_longs*)a)->data; }
static void f_rel_longs(JNIEnv* e, jlongArray a, jlong* p, jint m) { (void)e; (void)a; (void)p; (void)m; }
static jlongArray f_new_longs(JNIEnv* e, jsize n) {
    (void)e;
    fake_longs* b = (fake_longs*)calloc(1, sizeof(fake_longs) + (size_t)n * 8);
    b->len = n;
    return (jlongArray)b;
}
static void f_set_longs(JNIEnv* e, jlongArray a, jsize s, jsize n, const jlong* src) {
    (void)e;
    memcpy(((fake_longs*)a)->data + s, src, (size_t)n * 8);
}

static jobject f_new_direct(JNIEnv* e, void* a, jlong cap) { (void)e; (void)cap; return (jobject)a; }
static const struct JNINativeInterface_ g_table = {f_find_class, f_throw_new, f_direct, f_utf, f_rel_utf,
                                                   f_len, f_bytes, f_rel_bytes, f_new_bytes, f_set_region,
                                                   f_longs, f_rel_longs, f_new_longs, f_set_longs, f_new_direct};
static JNIEnv g_env = &g_table;

JNIEnv* fake_env(void) { return &g_env; }
jbyteArray fake_bytes_new(const void* data, jsize n) {
    jbyteArray a = f_new_bytes(&g_env, n);
    memcpy(((fake_bytes*)a)->data, data, (size_t)n);
    return a;
}
jsize fake_bytes_len(jbyteArray a) { return a ? ((fake_bytes*)a)->len : -1; }
const void* fake_bytes_data(jbyteArray a) { return ((fake_bytes*)a)->data; }
void fake_bytes_free(jbyteArray a) { free(a); }
int fake_exception(char* cls, char* msg, int cap) {
    int had = g_exc;
    if (had) {
        strncpy(cls, g_exc_class, (size_t)cap - 1);
        strncpy(msg, g_exc_msg, (size_t)cap - 1);
    }
    g_exc = 0;
    return had;
}
jlongArray fake_longs_new(const jlong* data, jsize n) {
    jlongArray a = f_new_longs(&g_env, n);
    memcpy(((fake_longs*)a)->data, data, (size_t)n * 8);
    return a;
}
const jlong* fake_longs_data(jlongArray a) { return ((fake_longs*)a)->data; }
