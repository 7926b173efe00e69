/* tests/jni_stub/fake_jvm.c — TEST ONLY.  A minimal JVM stand-in that fills
 * the JNIEnv function table of tests/jni_stub/jni.h, so that
 * tests/test_jni_gpu.py can EXECUTE every native method of
 * java/src/main/c/dbindex_jni.c (no JDK in this image) against
 * libdbindex_hip.so and read back exactly what the shim would hand to Java:
 * strings, primitive arrays, the SeqList object's fields, and the pending
 * exception (class + message).
 *
 * JNI rules it enforces (JNI specification, "JNI Functions"): no JNI call but
 * ExceptionCheck / DeleteLocalRef / ReleaseStringUTFChars while an exception
 * is pending (counted as violations), region accesses inside the array
 * (ArrayIndexOutOfBoundsException), every GetStringUTFChars released.
 * fj_fail_alloc_at(k) makes the k-th object allocation fail the way a JVM
 * does (NULL + a pending OutOfMemoryError). */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { FJ_CLASS = 1, FJ_STRING, FJ_BYTES, FJ_INTS, FJ_DOUBLES, FJ_OBJECT };
enum { FJ_MAX_FIELDS = 16 };

struct _jobject {
    int kind;
    char* name;      /* class name (FJ_CLASS, FJ_OBJECT), UTF-8 text (FJ_STRING) */
    void* data;      /* array elements */
    jsize len;       /* array length / string bytes */
    int nfields;
    const char* fname[FJ_MAX_FIELDS];
    jobject fval[FJ_MAX_FIELDS];
    struct _jobject* next_alloc;
};

struct _jfieldID {
    char name[64];
    char sig[16];
    struct _jfieldID* next_alloc;
};

static struct _jobject* g_objs = NULL;
static struct _jfieldID* g_fids = NULL;
static int g_pending = 0;
static char g_exc_class[256];
static char g_exc_msg[4096];
static int g_violations = 0;
static int g_utf_out = 0;  /* GetStringUTFChars not released yet */
static long g_allocs = 0, g_fail_at = -1;
static char g_log[8192];   /* FindClass names, in order */

static void violation_if_pending(const char* what) {
    if (g_pending) {
        ++g_violations;
        fprintf(stderr, "fake_jvm: %s called with an exception pending (%s)\n", what, g_exc_class);
    }
}

static void throw_class(const char* cls, const char* msg) {
    g_pending = 1;
    snprintf(g_exc_class, sizeof g_exc_class, "%s", cls);
    snprintf(g_exc_msg, sizeof g_exc_msg, "%s", msg ? msg : "");
}

/* one allocation of the JVM heap: NULL + OutOfMemoryError when injected */
static struct _jobject* new_obj(int kind) {
    if (g_fail_at >= 0 && g_allocs++ == g_fail_at) {
        throw_class("java/lang/OutOfMemoryError", "fake_jvm: injected allocation failure");
        return NULL;
    }
    struct _jobject* o = (struct _jobject*)calloc(1, sizeof(struct _jobject));
    if (!o) return NULL;
    o->kind = kind;
    o->next_alloc = g_objs;
    g_objs = o;
    return o;
}

static char* dup_str(const char* s) {
    const size_t n = strlen(s);
    char* d = (char*)malloc(n + 1);
    if (d) memcpy(d, s, n + 1);
    return d;
}

static jclass FindClass(JNIEnv* env, const char* name) {
    (void)env;
    violation_if_pending("FindClass");
    const size_t used = strlen(g_log), len = strlen(name);
    if (used + len + 2 <= sizeof g_log) {  /* the log keeps the first classes only */
        memcpy(g_log + used, name, len);
        g_log[used + len] = ';';
        g_log[used + len + 1] = 0;
    }
    struct _jobject* c = (struct _jobject*)calloc(1, sizeof(struct _jobject));
    c->kind = FJ_CLASS;
    c->name = dup_str(name);
    c->next_alloc = g_objs;
    g_objs = c;
    return c;
}

static jint ThrowNew(JNIEnv* env, jclass clazz, const char* msg) {
    (void)env;
    violation_if_pending("ThrowNew");
    throw_class(clazz && clazz->name ? clazz->name : "?", msg);
    return 0;
}

static jboolean ExceptionCheck(JNIEnv* env) {
    (void)env;
    return g_pending ? JNI_TRUE : JNI_FALSE;
}

static void DeleteLocalRef(JNIEnv* env, jobject obj) {
    (void)env;
    (void)obj; /* objects live until fj_reset */
}

static jobject AllocObject(JNIEnv* env, jclass clazz) {
    (void)env;
    violation_if_pending("AllocObject");
    struct _jobject* o = new_obj(FJ_OBJECT);
    if (o) o->name = dup_str(clazz->name);
    return o;
}

static jfieldID GetFieldID(JNIEnv* env, jclass clazz, const char* name, const char* sig) {
    (void)env;
    (void)clazz;
    violation_if_pending("GetFieldID");
    struct _jfieldID* f = (struct _jfieldID*)calloc(1, sizeof(struct _jfieldID));
    snprintf(f->name, sizeof f->name, "%s", name);
    snprintf(f->sig, sizeof f->sig, "%s", sig);
    f->next_alloc = g_fids;
    g_fids = f;
    return f;
}

static void SetObjectField(JNIEnv* env, jobject obj, jfieldID fid, jobject value) {
    (void)env;
    violation_if_pending("SetObjectField");
    if (!obj || obj->kind != FJ_OBJECT) {
        ++g_violations;
        return;
    }
    for (int i = 0; i < obj->nfields; ++i)
        if (strcmp(obj->fname[i], fid->name) == 0) {
            obj->fval[i] = value;
            return;
        }
    if (obj->nfields < FJ_MAX_FIELDS) {
        obj->fname[obj->nfields] = fid->name;
        obj->fval[obj->nfields++] = value;
    }
}

static jstring NewStringUTF(JNIEnv* env, const char* bytes) {
    (void)env;
    violation_if_pending("NewStringUTF");
    struct _jobject* o = new_obj(FJ_STRING);
    if (o) {
        o->name = dup_str(bytes);
        o->len = (jsize)strlen(bytes);
    }
    return o;
}

static const char* GetStringUTFChars(JNIEnv* env, jstring s, jboolean* isCopy) {
    (void)env;
    violation_if_pending("GetStringUTFChars");
    if (isCopy) *isCopy = JNI_TRUE;
    if (!s || s->kind != FJ_STRING) {
        ++g_violations;
        return NULL;
    }
    ++g_utf_out;
    return dup_str(s->name);
}

static void ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* utf) {
    (void)env;
    (void)s;
    --g_utf_out;
    free((void*)utf);
}

static jsize GetArrayLength(JNIEnv* env, jarray a) {
    (void)env;
    violation_if_pending("GetArrayLength");
    if (!a || a->kind < FJ_BYTES || a->kind > FJ_DOUBLES) {
        ++g_violations;
        return 0;
    }
    return a->len;
}

static jarray new_array(int kind, jsize n, size_t esz) {
    if (n < 0) {
        throw_class("java/lang/NegativeArraySizeException", "");
        return NULL;
    }
    struct _jobject* o = new_obj(kind);
    if (o) {
        o->len = n;
        o->data = calloc((size_t)n + 1, esz);
    }
    return o;
}

static jbyteArray NewByteArray(JNIEnv* env, jsize n) {
    (void)env;
    violation_if_pending("NewByteArray");
    return new_array(FJ_BYTES, n, 1);
}

static jintArray NewIntArray(JNIEnv* env, jsize n) {
    (void)env;
    violation_if_pending("NewIntArray");
    return new_array(FJ_INTS, n, 4);
}

static jdoubleArray NewDoubleArray(JNIEnv* env, jsize n) {
    (void)env;
    violation_if_pending("NewDoubleArray");
    return new_array(FJ_DOUBLES, n, 8);
}

/* region access: the array's kind and bounds, as the JVM checks them */
static int region_ok(jarray a, int kind, jsize start, jsize len) {
    if (!a || a->kind != kind) {
        ++g_violations;
        return 0;
    }
    if (start < 0 || len < 0 || start > a->len || len > a->len - start) {
        throw_class("java/lang/ArrayIndexOutOfBoundsException", "region");
        return 0;
    }
    return 1;
}

static void GetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize start, jsize len, jdouble* buf) {
    (void)env;
    violation_if_pending("GetDoubleArrayRegion");
    if (region_ok(a, FJ_DOUBLES, start, len)) memcpy(buf, (double*)a->data + start, 8 * (size_t)len);
}

static void SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize len, const jbyte* buf) {
    (void)env;
    violation_if_pending("SetByteArrayRegion");
    if (region_ok(a, FJ_BYTES, start, len)) memcpy((int8_t*)a->data + start, buf, (size_t)len);
}

static void SetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize len, const jint* buf) {
    (void)env;
    violation_if_pending("SetIntArrayRegion");
    if (region_ok(a, FJ_INTS, start, len)) memcpy((int32_t*)a->data + start, buf, 4 * (size_t)len);
}

static void SetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize start, jsize len, const jdouble* buf) {
    (void)env;
    violation_if_pending("SetDoubleArrayRegion");
    if (region_ok(a, FJ_DOUBLES, start, len)) memcpy((double*)a->data + start, buf, 8 * (size_t)len);
}

static const struct JNINativeInterface_ g_table = {
    FindClass,         ThrowNew,          ExceptionCheck,       DeleteLocalRef,       AllocObject,
    GetFieldID,        SetObjectField,    NewStringUTF,         GetStringUTFChars,    ReleaseStringUTFChars,
    GetArrayLength,    NewByteArray,      NewIntArray,          NewDoubleArray,       GetDoubleArrayRegion,
    SetByteArrayRegion, SetIntArrayRegion, SetDoubleArrayRegion,
};
static JNIEnv g_env = &g_table;

/* ---- the test's side (ctypes) ------------------------------------------- */
JNIEnv* fj_env(void) { return &g_env; }

jstring fj_string(const char* s) { return s ? NewStringUTF(&g_env, s) : NULL; }

jdoubleArray fj_doubles(const double* v, jsize n) {
    jdoubleArray a = new_array(FJ_DOUBLES, n, 8);
    if (a && n) memcpy(a->data, v, 8 * (size_t)n);
    return a;
}

int fj_kind(jobject o) { return o ? o->kind : 0; }
jsize fj_len(jobject o) { return o ? o->len : -1; }
const void* fj_data(jobject o) { return o ? o->data : NULL; }
const char* fj_name(jobject o) { return o ? o->name : NULL; }

jobject fj_field(jobject o, const char* name) {
    if (!o || o->kind != FJ_OBJECT) return NULL;
    for (int i = 0; i < o->nfields; ++i)
        if (strcmp(o->fname[i], name) == 0) return o->fval[i];
    return NULL;
}

/* the pending exception (class, message), cleared; 0 when none */
int fj_take_exception(char* cls, int ncls, char* msg, int nmsg) {
    const int p = g_pending;
    if (cls && ncls > 0) snprintf(cls, (size_t)ncls, "%s", p ? g_exc_class : "");
    if (msg && nmsg > 0) snprintf(msg, (size_t)nmsg, "%s", p ? g_exc_msg : "");
    g_pending = 0;
    return p;
}

int fj_violations(void) { return g_violations; }
int fj_utf_outstanding(void) { return g_utf_out; }
const char* fj_class_log(void) { return g_log; }

/* the k-th object allocation from now on fails (k < 0: none) */
void fj_fail_alloc_at(long k) {
    g_allocs = 0;
    g_fail_at = k;
}

void fj_reset(void) {
    while (g_objs) {
        struct _jobject* o = g_objs;
        g_objs = o->next_alloc;
        free(o->name);
        free(o->data);
        free(o);
    }
    while (g_fids) {
        struct _jfieldID* f = g_fids;
        g_fids = f->next_alloc;
        free(f);
    }
    g_pending = 0;
    g_violations = 0;
    g_utf_out = 0;
    g_fail_at = -1;
    g_allocs = 0;
    g_log[0] = 0;
}
