/* TEST-ONLY stand-in for the JDK's <jni.h>: declares just the JNI types and the JNIEnv
 * functions integration/jni/native/gw_jni.c uses, with their JNI-specification signatures,
 * so the glue compiles and runs here (no JDK in this image) against tests/jni/fake_env.c.
 * It is not ABI-compatible with a JVM's function table; a real build uses the JDK header. */
#ifndef GW_TEST_JNI_H
#define GW_TEST_JNI_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef double jdouble;
typedef jint jsize;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jlongArray;
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv* env, const char* name);
    jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
    const char* (*GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
    void (*ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
    jsize (*GetArrayLength)(JNIEnv* env, jarray array);
    jbyte* (*GetByteArrayElements)(JNIEnv* env, jbyteArray array, jboolean* isCopy);
    void (*ReleaseByteArrayElements)(JNIEnv* env, jbyteArray array, jbyte* elems, jint mode);
    jbyteArray (*NewByteArray)(JNIEnv* env, jsize len);
    void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
    jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray array, jboolean* isCopy);
    void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray array, jlong* elems, jint mode);
    jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
    void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
    jobject (*NewDirectByteBuffer)(JNIEnv* env, void* address, jlong capacity);
};
#endif
