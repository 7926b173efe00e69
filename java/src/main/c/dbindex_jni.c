/* dbindex_jni.c — JNI shim between edu.scripps.yates.dbindex.hip.DBIndexStoreHip
 * (DBIndexStore.java:19-194 on the MI355X engine) and libdbindex_hip.so.
 *
 * One native method = one dbi_store_* call of include/dbindex_hip.h; a
 * non-zero status becomes DBIndexStoreException(dbi_last_error()).  Nothing
 * is swallowed (the reference logs and continues, DBIndexer.java:398-403).
 *
 * Build (where a JDK exists; the image this repository is built in has none):
 *   make -C java        (java/Makefile)
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dbindex_hip.h"

#define JFN(name) Java_edu_scripps_yates_dbindex_hip_DBIndexStoreHip_##name
#define STORE(h) ((dbi_store*)(intptr_t)(h))

static const char* EXC = "edu/scripps/yates/utilities/fasta/dbindex/DBIndexStoreException";
static const char* SEQLIST = "edu/scripps/yates/dbindex/hip/DBIndexStoreHip$SeqList";

/* status -> pending checked exception; returns rc.  An exception already
 * pending (an OutOfMemoryError of a JNI call) is left as it is: JNI allows no
 * further throw while one is pending. */
static int fail(JNIEnv* e, int rc) {
    if (rc && !(*e)->ExceptionCheck(e)) {
        jclass c = (*e)->FindClass(e, EXC);
        if (c) (*e)->ThrowNew(e, c, dbi_last_error());
    }
    return rc;
}

/* a malloc of the shim failed (a failed JNI allocation has thrown already) */
static int oom(JNIEnv* e) {
    if (!(*e)->ExceptionCheck(e)) {
        jclass c = (*e)->FindClass(e, "java/lang/OutOfMemoryError");
        if (c) (*e)->ThrowNew(e, c, "dbindex_jni");
    }
    return DBI_E_OOM;
}

/* chars of a Java string into flag table t (1 per residue present); -1 when
 * the JVM could not copy the string (OutOfMemoryError pending) */
static int residue_flags(JNIEnv* e, jstring s, uint8_t* t) {
    memset(t, 0, 256);
    if (!s) return 0;
    const char* c = (*e)->GetStringUTFChars(e, s, NULL);
    if (!c) return -1;
    for (const char* p = c; *p; ++p) t[(unsigned char)*p] = 1;
    (*e)->ReleaseStringUTFChars(e, s, c);
    return 0;
}

JNIEXPORT jlong JNICALL JFN(create)(JNIEnv* e, jclass k, jdoubleArray mass, jstring cleave, jstring nocut,
                                    jstring mandatory, jint maxMissed, jboolean semi, jdouble minMH,
                                    jdouble maxMH, jboolean addH2O, jdouble h2oProton, jdouble cTerm,
                                    jdouble nTerm, jint factor, jint indexFactor, jint device) {
    (void)k;
    dbi_params p;
    dbi_params_default(&p, maxMissed, semi ? 1 : 0);
    if ((*e)->GetArrayLength(e, mass) != 256) {
        jclass c = (*e)->FindClass(e, EXC);
        if (c) (*e)->ThrowNew(e, c, "mass table must hold 256 entries");
        return 0;
    }
    (*e)->GetDoubleArrayRegion(e, mass, 0, 256, p.mass);   /* AssignMass.getMass(c), every c */
    if (residue_flags(e, cleave, p.cleave) ||              /* Enzyme residues               */
        residue_flags(e, nocut, p.nocut) ||                /* getEnzymeNocutResidues()      */
        residue_flags(e, mandatory, p.mandatory))          /* getMandatoryInternalAAs()     */
        return 0;
    p.mandatory_mode = mandatory != NULL;                  /* null vs empty (DBIndexer.java:334) */
    p.mandatory_count = 0;
    for (int c = 0; c < 256; ++c) p.mandatory_count += p.mandatory[c];
    p.min_mh = minMH;
    p.max_mh = maxMH;
    p.add_h2o_proton = addH2O ? 1 : 0;
    p.h2o_proton = h2oProton;
    p.cterm = cTerm;
    p.nterm = nTerm;
    p.mass_group_factor = factor;
    p.index_factor = indexFactor;
    dbi_store* st = NULL;
    if (fail(e, dbi_store_create(&p, device, &st))) return 0;
    return (jlong)(intptr_t)st;
}

JNIEXPORT void JNICALL JFN(close0)(JNIEnv* e, jclass k, jlong h) {
    (void)e; (void)k;
    dbi_store_close(STORE(h));
}

JNIEXPORT void JNICALL JFN(init0)(JNIEnv* e, jclass k, jlong h, jstring id) {
    (void)k;
    const char* s = id ? (*e)->GetStringUTFChars(e, id, NULL) : NULL;
    if (id && !s) return; /* OutOfMemoryError pending */
    const int rc = dbi_store_init(STORE(h), s ? s : "");
    if (s) (*e)->ReleaseStringUTFChars(e, id, s);
    fail(e, rc);
}

JNIEXPORT void JNICALL JFN(startAddSeq0)(JNIEnv* e, jclass k, jlong h) {
    (void)k;
    fail(e, dbi_store_start_add_seq(STORE(h)));
}

JNIEXPORT void JNICALL JFN(stopAddSeq0)(JNIEnv* e, jclass k, jlong h) {
    (void)k;
    fail(e, dbi_store_stop_add_seq(STORE(h)));  /* the GPU digest + sort + merge happen here */
}

JNIEXPORT jboolean JNICALL JFN(indexExists0)(JNIEnv* e, jclass k, jlong h) {
    (void)k;
    int out = 0;
    if (fail(e, dbi_store_index_exists(STORE(h), &out))) return JNI_FALSE;
    return out ? JNI_TRUE : JNI_FALSE;
}

JNIEXPORT jint JNICALL JFN(filterSequence0)(JNIEnv* e, jclass k, jlong h, jdouble mass, jstring seq) {
    (void)k;
    const char* s = (*e)->GetStringUTFChars(e, seq, NULL);
    int out = DBI_FILTER_SKIP;
    if (!s) return out; /* OutOfMemoryError pending */
    const int rc = dbi_store_filter_sequence(STORE(h), mass, s, strlen(s), &out);
    (*e)->ReleaseStringUTFChars(e, seq, s);
    fail(e, rc);  /* filterSequence declares no exception: an unchecked-style pending one */
    return out;
}

JNIEXPORT void JNICALL JFN(addSequence0)(JNIEnv* e, jclass k, jlong h, jdouble mass, jint offset, jint length,
                                         jlong proteinId) {
    (void)k;
    fail(e, dbi_store_add_sequence(STORE(h), mass, offset, length, proteinId));
}

JNIEXPORT jlong JNICALL JFN(addProteinDef0)(JNIEnv* e, jclass k, jlong h, jlong num, jstring def, jstring seq) {
    (void)k;
    const char* d = (*e)->GetStringUTFChars(e, def, NULL);
    if (!d) return -1; /* OutOfMemoryError pending */
    const char* q = (*e)->GetStringUTFChars(e, seq, NULL);
    if (!q) {
        (*e)->ReleaseStringUTFChars(e, def, d);
        return -1;
    }
    int64_t id = -1;
    const int rc = dbi_store_add_protein_def(STORE(h), num, d, q, strlen(q), &id);
    (*e)->ReleaseStringUTFChars(e, def, d);
    (*e)->ReleaseStringUTFChars(e, seq, q);
    fail(e, rc);
    return id;
}

JNIEXPORT jlong JNICALL JFN(getNumberSequences0)(JNIEnv* e, jclass k, jlong h) {
    (void)k;
    int64_t n = 0;
    fail(e, dbi_store_get_number_sequences(STORE(h), &n));
    return n;
}

JNIEXPORT jlong JNICALL JFN(getTotalSeqCount0)(JNIEnv* e, jclass k, jlong h) {
    (void)k;
    int64_t n = 0;
    fail(e, dbi_store_get_total_seq_count(STORE(h), &n));
    return n;
}

JNIEXPORT jintArray JNICALL JFN(getEntryKeys0)(JNIEnv* e, jclass k, jlong h) {
    (void)k;
    uint64_t n = 0;
    if (fail(e, dbi_store_get_entry_keys(STORE(h), NULL, 0, &n))) return NULL;
    int32_t* keys = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
    if (!keys) return oom(e), NULL;
    if (fail(e, dbi_store_get_entry_keys(STORE(h), keys, n, &n))) {
        free(keys);
        return NULL;
    }
    jintArray a = (*e)->NewIntArray(e, (jsize)n);
    if (a) (*e)->SetIntArrayRegion(e, a, 0, (jsize)n, (const jint*)keys);
    free(keys);
    return a;
}

static jstring protein_string(JNIEnv* e, int rc, const char* s, uint64_t len) {
    if (fail(e, rc)) return NULL;
    char* z = (char*)malloc(len + 1);
    if (!z) return oom(e), NULL;
    memcpy(z, s, len);
    z[len] = 0;
    jstring r = (*e)->NewStringUTF(e, z);
    free(z);
    return r;
}

JNIEXPORT jstring JNICALL JFN(proteinDef0)(JNIEnv* e, jclass k, jlong h, jlong id) {
    (void)k;
    const char* s = NULL;
    uint64_t len = 0;
    const int rc = dbi_store_protein_def(STORE(h), (uint64_t)id, &s, &len);
    return protein_string(e, rc, s, len);
}

JNIEXPORT jstring JNICALL JFN(proteinSequence0)(JNIEnv* e, jclass k, jlong h, jlong id) {
    (void)k;
    const char* s = NULL;
    uint64_t len = 0;
    const int rc = dbi_store_protein_sequence(STORE(h), (uint64_t)id, &s, &len);
    return protein_string(e, rc, s, len);
}

JNIEXPORT void JNICALL JFN(setDeviceDigest0)(JNIEnv* e, jclass k, jlong h, jboolean on) {
    (void)k;
    fail(e, dbi_store_set_device_digest(STORE(h), on ? 1 : 0));
}

JNIEXPORT void JNICALL JFN(setPersist0)(JNIEnv* e, jclass k, jlong h, jboolean on) {
    (void)k;
    fail(e, dbi_store_set_persist(STORE(h), on ? 1 : 0));
}

JNIEXPORT void JNICALL JFN(setUnindexed0)(JNIEnv* e, jclass k, jlong h, jint mode) {
    (void)k;
    fail(e, dbi_store_set_unindexed(STORE(h), mode));
}

/* dbi_seq_list -> DBIndexStoreHip.SeqList (flat arrays; Java builds the
 * IndexedSequence objects, DBIndexStoreHip.toList) */
static int set_array(JNIEnv* e, jobject o, jclass c, const char* name, const char* sig, jobject arr) {
    if (!arr) return DBI_E_OOM; /* the failed New<Type>Array threw OutOfMemoryError */
    jfieldID f = (*e)->GetFieldID(e, c, name, sig);
    if (!f) return DBI_E_INVALID;
    (*e)->SetObjectField(e, o, f, arr);
    (*e)->DeleteLocalRef(e, arr);
    return 0;
}

static jobject seq_list(JNIEnv* e, dbi_seq_list* l) {
    jclass c = (*e)->FindClass(e, SEQLIST);
    if (!c) return NULL;
    jobject o = (*e)->AllocObject(e, c);
    if (!o) return NULL;
    const jsize n = (jsize)l->n;
    const jsize nc = (jsize)l->seq_off[l->n], np = (jsize)l->prot_off[l->n];
    jint* so = (jint*)malloc(sizeof(jint) * (size_t)(n + 1));
    jint* po = (jint*)malloc(sizeof(jint) * (size_t)(n + 1));
    if (!so || !po) {
        free(so);
        free(po);
        return oom(e), NULL;
    }
    for (jsize i = 0; i <= n; ++i) {
        so[i] = (jint)l->seq_off[i];
        po[i] = (jint)l->prot_off[i];
    }
    /* one JVM allocation at a time: after a failed one (OutOfMemoryError
     * pending) no further JNI call but the cleanup (JNI specification) */
    jobject ret = NULL;
    jdoubleArray mass = NULL;
    jintArray seqOff = NULL, protOff = NULL, protIds = NULL, pepOff = NULL;
    jbyteArray chars = NULL, left = NULL, right = NULL;
    if (!(mass = (*e)->NewDoubleArray(e, n))) goto done;
    (*e)->SetDoubleArrayRegion(e, mass, 0, n, l->mass);
    if (!(seqOff = (*e)->NewIntArray(e, n + 1))) goto done;
    (*e)->SetIntArrayRegion(e, seqOff, 0, n + 1, so);
    if (!(chars = (*e)->NewByteArray(e, nc))) goto done;
    (*e)->SetByteArrayRegion(e, chars, 0, nc, (const jbyte*)l->seq_chars);
    if (!(left = (*e)->NewByteArray(e, 3 * n))) goto done;
    (*e)->SetByteArrayRegion(e, left, 0, 3 * n, (const jbyte*)l->res_left);
    if (!(right = (*e)->NewByteArray(e, 3 * n))) goto done;
    (*e)->SetByteArrayRegion(e, right, 0, 3 * n, (const jbyte*)l->res_right);
    if (!(protOff = (*e)->NewIntArray(e, n + 1))) goto done;
    (*e)->SetIntArrayRegion(e, protOff, 0, n + 1, po);
    if (!(protIds = (*e)->NewIntArray(e, np))) goto done;
    (*e)->SetIntArrayRegion(e, protIds, 0, np, (const jint*)l->prot_ids);
    if (!(pepOff = (*e)->NewIntArray(e, n))) goto done;
    (*e)->SetIntArrayRegion(e, pepOff, 0, n, (const jint*)l->offset);
    if (set_array(e, o, c, "mass", "[D", mass) || set_array(e, o, c, "seqOff", "[I", seqOff) ||
        set_array(e, o, c, "seqChars", "[B", chars) || set_array(e, o, c, "left", "[B", left) ||
        set_array(e, o, c, "right", "[B", right) || set_array(e, o, c, "protOff", "[I", protOff) ||
        set_array(e, o, c, "protIds", "[I", protIds) || set_array(e, o, c, "pepOff", "[I", pepOff))
        goto done;
    ret = o;
done:
    free(so);
    free(po);
    return ret;
}

static jobject finish_list(JNIEnv* e, int rc, dbi_seq_list* l) {
    if (fail(e, rc)) return NULL;
    jobject o = seq_list(e, l);
    dbi_seq_list_free(l);
    return o;
}

JNIEXPORT jobject JNICALL JFN(getSequences0)(JNIEnv* e, jclass k, jlong h, jdouble mass, jdouble tol) {
    (void)k;
    dbi_seq_list* l = NULL;
    const int rc = dbi_store_get_sequences(STORE(h), mass, tol, &l);
    return finish_list(e, rc, l);
}

/* two double[] of one length into malloc'd copies */
static int ranges_of(JNIEnv* e, jdoubleArray m, jdoubleArray t, double** mo, double** to, uint64_t* n) {
    const jsize k = (*e)->GetArrayLength(e, m);
    if ((*e)->GetArrayLength(e, t) != k) {
        jclass c = (*e)->FindClass(e, EXC);
        if (c) (*e)->ThrowNew(e, c, "mass and tolerance arrays differ in length");
        return DBI_E_INVALID;
    }
    *mo = (double*)malloc(sizeof(double) * (size_t)(k ? k : 1));
    *to = (double*)malloc(sizeof(double) * (size_t)(k ? k : 1));
    if (!*mo || !*to) {
        free(*mo);
        free(*to);
        return oom(e);
    }
    (*e)->GetDoubleArrayRegion(e, m, 0, k, *mo);
    (*e)->GetDoubleArrayRegion(e, t, 0, k, *to);
    *n = (uint64_t)k;
    return 0;
}

JNIEXPORT jobject JNICALL JFN(getSequencesRanges0)(JNIEnv* e, jclass k, jlong h, jdoubleArray m, jdoubleArray t) {
    (void)k;
    double *mo, *to;
    uint64_t n;
    if (ranges_of(e, m, t, &mo, &to, &n)) return NULL;
    dbi_seq_list* l = NULL;
    const int rc = dbi_store_get_sequences_ranges(STORE(h), mo, to, n, &l);
    free(mo);
    free(to);
    return finish_list(e, rc, l);
}

JNIEXPORT jobject JNICALL JFN(cutAndSearch0)(JNIEnv* e, jclass k, jlong h, jdoubleArray m, jdoubleArray t) {
    (void)k;
    double *mo, *to;
    uint64_t n;
    if (ranges_of(e, m, t, &mo, &to, &n)) return NULL;
    dbi_seq_list* l = NULL;
    const int rc = dbi_store_cut_and_search(STORE(h), mo, to, n, &l);
    free(mo);
    free(to);
    return finish_list(e, rc, l);
}
