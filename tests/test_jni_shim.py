"""CPU checks of the Java/JNI drop-in (java/): no JDK exists in this image, so
the shim is checked structurally — every dbi_* function the JNI C file calls
is declared in include/dbindex_hip.h with the same number of arguments, and
every native method of DBIndexStoreHip.java has its JNI definition with the
matching arity (JNIEnv* and jclass first).  Reference: DBIndexStore.java:19-194,
DBIndexer.java:143-155,237."""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "java", "src", "main", "c", "dbindex_jni.c")
JAVA = os.path.join(ROOT, "java", "src", "main", "java", "edu", "scripps", "yates", "dbindex", "hip")
HEADER = os.path.join(ROOT, "include", "dbindex_hip.h")


def _strip_comments(s: str) -> str:
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def _split_args(args: str):
    depth, cur, out = 0, "", []
    for ch in args:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out if a.strip() and a.strip() != "void"]


def _header_arity():
    h = _strip_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"\b(dbi_\w+)\s*\(([^;{]*?)\)\s*;", h, flags=re.S):
        out[m.group(1)] = len(_split_args(m.group(2)))
    return out


def _calls(src: str):
    """(name, argument count) of every dbi_* call (balanced parentheses)."""
    out = []
    for m in re.finditer(r"\b(dbi_[a-z_0-9]+)\s*\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        out.append((m.group(1), len(_split_args(src[m.end():i - 1]))))
    return out


def test_jni_calls_match_header():
    decl = _header_arity()
    src = _strip_comments(open(JNI).read())
    calls = _calls(src)
    assert len(calls) >= 20
    for name, n in calls:
        assert name in decl, f"{name} is not declared in include/dbindex_hip.h"
        assert n == decl[name], f"{name}: {n} arguments in the shim, {decl[name]} in the header"
    # every store entry point of the DBIndexStore mirror is bound
    bound = {n for n, _ in calls}
    for name in decl:
        # engine view / protein count: batch-path helpers the Java store does not need
        if name.startswith("dbi_store_") and name not in ("dbi_store_engine", "dbi_store_protein_count"):
            assert name in bound, f"{name} has no JNI binding"


def test_every_native_method_has_a_jni_definition():
    java = open(os.path.join(JAVA, "DBIndexStoreHip.java")).read()
    natives = {}
    for m in re.finditer(r"native\s+[\w\[\]<>.]+\s+(\w+)\s*\(([^)]*)\)", java):
        natives[m.group(1)] = len(_split_args(m.group(2)))
    assert len(natives) >= 18
    src = _strip_comments(open(JNI).read())
    for name, n in natives.items():
        m = re.search(r"JFN\(" + name + r"\)\s*\(([^)]*)\)", src)
        assert m, f"native {name} has no JNI definition"
        assert len(_split_args(m.group(1))) == n + 2, f"{name}: arity"


def test_java_side_overrides_the_reference_interface():
    """DBIndexStoreHip implements every DBIndexStore method the reference declares
    (DBIndexStore.java:19-194), and DBIndexerHip overrides the protected cutSeq."""
    store = open(os.path.join(JAVA, "DBIndexStoreHip.java")).read()
    for meth in ("init", "startAddSeq", "stopAddSeq", "indexExists", "filterSequence", "addSequence",
                 "getSequences", "getSequencesIterator", "addProteinDef", "setProteinCache",
                 "supportsProteinCache", "getProteins", "getNumberSequences", "getResidues", "getEntryKeys",
                 "lastBuffertoDatabase"):
        assert re.search(r"public\s+[\w<>\[\]. ]+\s+" + meth + r"\s*\(", store), meth
    assert "implements DBIndexStore" in store
    idx = open(os.path.join(JAVA, "DBIndexerHip.java")).read()
    assert "extends DBIndexer" in idx and re.search(r"protected void cutSeq\(", idx)
    # SEARCH_UNINDEXED queries bypass the private cutAndSearch (DBIndexer.java:707-747)
    for meth in ("getSequencesUsingDaltonTolerance", "getSequencesUsingPPMTolerance", "getSequences"):
        assert re.search(r"@Override\s+public List<IndexedSequence> " + meth + r"\(", idx), meth
    assert re.search(r"public List<IndexedSequence> cutAndSearch\(List<MassRange>", store)
    impl = open(os.path.join(JAVA, "DBIndexImplHip.java")).read()
    assert "extends DBIndexImpl" in impl and "new DBIndexerHip(" in impl


STUB = os.path.join(ROOT, "tests", "jni_stub")


def test_jni_shim_compiles_against_the_header():
    """The shim passes a C compiler with every warning an error: each
    dbi_store_* call is type-checked against include/dbindex_hip.h (types,
    not just arity).  The JNI types come from a test-only header declaring
    the specification's C signatures of the JNIEnv entries the shim uses
    (tests/jni_stub/jni.h: no JDK in this image)."""
    import subprocess
    r = subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Wextra", "-Werror", "-Wconversion",
                        "-Wno-sign-conversion", "-Wstrict-prototypes", "-I", STUB, "-I", os.path.join(ROOT, "include"),
                        JNI], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_jni_shim_links_against_the_library(tmp_path):
    """Linked as the JNI library a JVM would load: every dbi_* symbol the
    shim calls resolves in the built libdbindex_hip.so (--no-undefined)."""
    import subprocess
    import pytest
    lib = os.path.join(ROOT, "dbindex_amd", "libdbindex_hip.so")
    if not os.path.exists(lib):
        pytest.skip("libdbindex_hip.so not built")
    out = tmp_path / "libdbindex_jni.so"
    r = subprocess.run(["gcc", "-shared", "-fPIC", "-std=c11", "-O2", "-I", STUB, "-I", os.path.join(ROOT, "include"),
                        JNI, "-o", str(out), "-L", os.path.dirname(lib), "-l:libdbindex_hip.so",
                        "-Wl,--no-undefined", f"-Wl,-rpath,{os.path.dirname(lib)}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", "-D", "--defined-only", str(out)], capture_output=True, text=True).stdout
    assert "Java_edu_scripps_yates_dbindex_hip_DBIndexStoreHip_getSequences0" in nm
