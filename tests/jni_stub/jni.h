/* tests/jni_stub/jni.h — TEST ONLY.  The image has no JDK, so this declares
 * just the part of the JNI C API (JNI specification, "JNI Functions": types,
 * the JNIEnv function table entries) that java/src/main/c/dbindex_jni.c uses,
 * with the specification's C signatures, so that tests/test_jni_shim.py can
 * compile the shim with -Werror and type-check every dbi_store_* call against
 * include/dbindex_hip.h.  The real header replaces it in a maintainer's build
 * (java/Makefile). */
#ifndef DBINDEX_TEST_JNI_STUB_H
#define DBINDEX_TEST_JNI_STUB_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1

typedef uint8_t jboolean;
typedef int8_t jbyte;
typedef int32_t jint;
typedef int64_t jlong;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jdoubleArray;
struct _jfieldID;
typedef struct _jfieldID* jfieldID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv* env, const char* name);
    jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    jboolean (*ExceptionCheck)(JNIEnv* env);
    void (*DeleteLocalRef)(JNIEnv* env, jobject obj);
    jobject (*AllocObject)(JNIEnv* env, jclass clazz);
    jfieldID (*GetFieldID)(JNIEnv* env, jclass clazz, const char* name, const char* sig);
    void (*SetObjectField)(JNIEnv* env, jobject obj, jfieldID fieldID, jobject value);
    jstring (*NewStringUTF)(JNIEnv* env, const char* bytes);
    const char* (*GetStringUTFChars)(JNIEnv* env, jstring string, jboolean* isCopy);
    void (*ReleaseStringUTFChars)(JNIEnv* env, jstring string, const char* utf);
    jsize (*GetArrayLength)(JNIEnv* env, jarray array);
    jbyteArray (*NewByteArray)(JNIEnv* env, jsize length);
    jintArray (*NewIntArray)(JNIEnv* env, jsize length);
    jdoubleArray (*NewDoubleArray)(JNIEnv* env, jsize length);
    void (*GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, jdouble* buf);
    void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
    void (*SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf);
    void (*SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
};
#endif
