"""The JNI shim EXECUTED on the CPU: the natives of DBIndexStoreHip whose
store calls need no device (create, init, addProteinDef, filterSequence,
addSequence, the ProteinCache strings, every error path before a build) run
through the fake JVM of tests/jni_stub/fake_jvm.c against
libdbindex_hip.so.  Builds and queries run on the GPU (test_jni_gpu.py).

Reference: DBIndexStore.java:37-192; DBIndexStoreSQLiteMult.java:245-291
(filterSequence / addSequence), :92-149 (init)."""
from __future__ import annotations

import numpy as np
import pytest

from dbindex_amd.params import DBIndexSearchParams
from tests.jni_stub.harness import EXC, JavaException, Jvm, JniStore


@pytest.fixture(scope="module")
def jvm():
    j = Jvm()
    yield j
    j.reset()


def last_error() -> str:
    from dbindex_amd import _native
    return _native.lib().dbi_last_error().decode()


def clean(j):
    assert j.violations() == 0, "a JNI call was made with an exception pending"
    assert j.utf_outstanding() == 0, "GetStringUTFChars without ReleaseStringUTFChars"


def test_jni_errors_become_dbindexstoreexception(jvm):
    """A non-zero status of any dbi_store_* call is a pending
    DBIndexStoreException carrying dbi_last_error(); the shim makes no JNI
    call while an exception is pending and releases every UTF string."""
    cp = DBIndexSearchParams.trypsin(2).to_c()
    st = JniStore(jvm, cp)
    try:
        # calls before init: the store's state errors (DBIndexStoreSQLiteMult's
        # "Indexer is not initialized")
        with pytest.raises(JavaException) as ei:
            st.getSequences(1000.0, 0.1)
        assert ei.value.cls == EXC and ei.value.msg == last_error() and "not initialized" in ei.value.msg
        with pytest.raises(JavaException) as ei:
            st.getNumberSequences()
        assert ei.value.cls == EXC and ei.value.msg == last_error()
        with pytest.raises(JavaException) as ei:
            st.stopAddSeq()
        assert ei.value.cls == EXC and ei.value.msg == last_error()
        st.init("errors.fasta")
        # arrays of different lengths: thrown by the shim itself
        with pytest.raises(JavaException) as ei:
            st.ranges("getSequencesRanges0", [1000.0, 1100.0], [0.1])
        assert ei.value.cls == EXC and "differ in length" in ei.value.msg
        st.startAddSeq()
        # protein numbers out of FASTA order
        with pytest.raises(JavaException) as ei:
            st.addProteinDef(5, "sp|P5|X", "PEPTIDEK")
        assert ei.value.cls == EXC and ei.value.msg == last_error()
        assert st.addProteinDef(0, "sp|P1|X", "PEPTIDEKAAAAAAR") == 0
        # an occurrence outside its protein; an unknown protein id
        with pytest.raises(JavaException) as ei:
            st.addSequence(1000.0, 10, 9, 0)
        assert ei.value.cls == EXC and ei.value.msg == last_error() and "outside" in ei.value.msg
        with pytest.raises(JavaException) as ei:
            st.addSequence(1000.0, 0, 3, 7)
        assert ei.value.cls == EXC and ei.value.msg == last_error()
        st.addSequence(927.4, 0, 8, 0)
        st.addSequence(9000.0, 0, 8, 0)  # bucket past NUM_BUCKETS-1: counted, not stored
        assert st.getTotalSeqCount() == 4  # every addSequence call counts (SQLiteMult.java:277)
        # the device digest cannot take over a transaction that holds occurrences
        with pytest.raises(JavaException) as ei:
            st.setDeviceDigest(True)
        assert ei.value.cls == EXC and ei.value.msg == last_error()
        # with it on (a fresh store), addSequence refuses: occurrences come from the GPU
        st2 = JniStore(jvm, cp)
        try:
            st2.setDeviceDigest(True)
            st2.init("errors2.fasta")
            with pytest.raises(JavaException) as ei:
                st2.addSequence(1000.0, 0, 3, 0)
            assert ei.value.cls == EXC and ei.value.msg == last_error()
        finally:
            st2.close()
        clean(jvm)
    finally:
        st.close()
    # create with a mass table that is not 256 long
    with pytest.raises(JavaException) as ei:
        jvm.call("create", jvm.doubles(np.zeros(255)), jvm.string("KR"), jvm.string(""), None, 2, 0, 500.0,
                 6000.0, 1, 19.0, 0.0, 0.0, 10000, 8, 0)
    assert ei.value.cls == EXC and "256" in ei.value.msg
    # invalid parameters: dbi_store_create's own status
    with pytest.raises(JavaException) as ei:
        jvm.call("create", jvm.doubles(np.array(cp.mass[:])), jvm.string("KR"), jvm.string(""), None, 2, 0,
                 500.0, 6000.0, 1, 19.0, 0.0, 0.0, 10000, 0, 0)
    assert ei.value.cls == EXC and ei.value.msg == last_error() and "index_factor" in ei.value.msg
    clean(jvm)
    jvm.reset()


    jvm.reset()


def test_jni_host_natives(jvm):
    """create / init / addProteinDef / the ProteinCache strings /
    filterSequence: the values the natives hand back to Java."""
    prm = DBIndexSearchParams.trypsin(2)
    st = JniStore(jvm, prm.to_c())
    try:
        st.init("host.fasta")
        assert st.indexExists() == 0
        st.startAddSeq()
        prots = [("sp|P1|A\tdef", "PEPTIDEKAAAAAAR"), ("sp|P2|B", "MKWVTFISLLLLFSSAYS")]
        for i, (d, q) in enumerate(prots):
            assert st.addProteinDef(i, d, q) == i
        assert jvm.read(st.proteinDef(0)) == "sp|P1|A\tdef".replace("\t", " ")  # ProteinCache.addProtein (:87-89)
        assert jvm.read(st.proteinSequence(1)) == prots[1][1]
        with pytest.raises(JavaException) as ei:
            st.proteinSequence(2)
        assert ei.value.cls == EXC and ei.value.msg == last_error()
        # filterSequence: INCLUDE inside [minMH, maxMH], SKIP outside (SQLiteMult.java:245-268)
        assert st.filterSequence(927.4, "PEPTIDEK") == 0
        assert st.filterSequence(499.9, "PEPTIDEK") == 1 and st.filterSequence(6000.1, "PEPTIDEK") == 1
        keys = jvm.read(st.getEntryKeys())
        assert keys.shape == (0,)
        clean(jvm)
        for k in range(2):  # the String of a definition; the int[] of the keys
            jvm.fail_alloc_at(0)
            with pytest.raises(JavaException) as ei:
                (st.proteinDef if k == 0 else (lambda _x: st.getEntryKeys()))(0)
            assert ei.value.cls == "java/lang/OutOfMemoryError"
            clean(jvm)
        jvm.fail_alloc_at(-1)
    finally:
        st.close()
        jvm.reset()
