"""TEST ONLY: builds and drives the JNI shim (java/src/main/c/dbindex_jni.c)
inside the fake JVM of tests/jni_stub/fake_jvm.c, so the native methods of
DBIndexStoreHip run for real against libdbindex_hip.so without a JDK.

``JniStore`` mirrors the ``private static native`` methods of
DBIndexStoreHip.java one for one: each call passes the fake JNIEnv and a NULL
jclass, then turns a pending Java exception into ``JavaException`` (class,
message) -- what the JVM would raise in the Java caller."""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_long, c_uint8, c_void_p
from typing import Dict, List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SHIM = os.path.join(ROOT, "java", "src", "main", "c", "dbindex_jni.c")
FAKE = os.path.join(HERE, "fake_jvm.c")
LIBDIR = os.path.join(ROOT, "dbindex_amd")
OUT = os.path.join(HERE, "build", "libjni_harness.so")
PREFIX = "Java_edu_scripps_yates_dbindex_hip_DBIndexStoreHip_"
EXC = "edu/scripps/yates/utilities/fasta/dbindex/DBIndexStoreException"

FJ_CLASS, FJ_STRING, FJ_BYTES, FJ_INTS, FJ_DOUBLES, FJ_OBJECT = range(1, 7)


def build(force: bool = False) -> str:
    """gcc: the shim + the fake JVM, linked against the built library."""
    deps = [SHIM, FAKE, os.path.join(HERE, "jni.h"), os.path.join(ROOT, "include", "dbindex_hip.h"),
            os.path.join(LIBDIR, "libdbindex_hip.so")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(d) <= os.path.getmtime(OUT) for d in deps):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + ".tmp"
    r = subprocess.run(["gcc", "-shared", "-fPIC", "-std=c11", "-O1", "-g", "-Wall", "-Wextra", "-Werror",
                        "-I", HERE, "-I", os.path.join(ROOT, "include"), SHIM, FAKE, "-o", tmp,
                        "-L", LIBDIR, "-l:libdbindex_hip.so", "-Wl,--no-undefined", f"-Wl,-rpath,{LIBDIR}"],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"JNI harness build failed:\n{r.stderr}")
    os.replace(tmp, OUT)
    return OUT


class JavaException(Exception):
    def __init__(self, cls: str, msg: str):
        super().__init__(f"{cls}: {msg}")
        self.cls, self.msg = cls, msg


_NATIVES = {  # name: (restype, argtypes after (JNIEnv*, jclass)) -- DBIndexStoreHip.java:297-343
    "create": (c_int64, [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_uint8, c_double, c_double, c_uint8,
                         c_double, c_double, c_double, c_int32, c_int32, c_int32]),
    "close0": (None, [c_int64]),
    "init0": (None, [c_int64, c_void_p]),
    "startAddSeq0": (None, [c_int64]),
    "stopAddSeq0": (None, [c_int64]),
    "indexExists0": (c_uint8, [c_int64]),
    "filterSequence0": (c_int32, [c_int64, c_double, c_void_p]),
    "addSequence0": (None, [c_int64, c_double, c_int32, c_int32, c_int64]),
    "getSequences0": (c_void_p, [c_int64, c_double, c_double]),
    "getSequencesRanges0": (c_void_p, [c_int64, c_void_p, c_void_p]),
    "cutAndSearch0": (c_void_p, [c_int64, c_void_p, c_void_p]),
    "addProteinDef0": (c_int64, [c_int64, c_int64, c_void_p, c_void_p]),
    "getNumberSequences0": (c_int64, [c_int64]),
    "getTotalSeqCount0": (c_int64, [c_int64]),
    "getEntryKeys0": (c_void_p, [c_int64]),
    "proteinDef0": (c_void_p, [c_int64, c_int64]),
    "proteinSequence0": (c_void_p, [c_int64, c_int64]),
    "setDeviceDigest0": (None, [c_int64, c_uint8]),
    "setPersist0": (None, [c_int64, c_uint8]),
    "setUnindexed0": (None, [c_int64, c_int32]),
}


class Jvm:
    """The loaded harness: JNIEnv, object constructors / readers, natives."""

    def __init__(self, path: Optional[str] = None):
        from dbindex_amd import _native
        _native.lib()  # the engine library first (its runtime checks)
        L = ctypes.CDLL(path or build())
        self.L = L
        L.fj_env.restype = c_void_p
        L.fj_string.restype = c_void_p
        L.fj_string.argtypes = [c_char_p]
        L.fj_doubles.restype = c_void_p
        L.fj_doubles.argtypes = [c_void_p, c_int]
        for f in ("fj_kind", "fj_len"):
            getattr(L, f).restype = c_int
            getattr(L, f).argtypes = [c_void_p]
        L.fj_data.restype = c_void_p
        L.fj_data.argtypes = [c_void_p]
        L.fj_name.restype = c_char_p
        L.fj_name.argtypes = [c_void_p]
        L.fj_field.restype = c_void_p
        L.fj_field.argtypes = [c_void_p, c_char_p]
        L.fj_take_exception.restype = c_int
        L.fj_take_exception.argtypes = [c_char_p, c_int, c_char_p, c_int]
        L.fj_violations.restype = c_int
        L.fj_utf_outstanding.restype = c_int
        L.fj_class_log.restype = c_char_p
        L.fj_fail_alloc_at.argtypes = [c_long]
        self.env = L.fj_env()
        self.fn: Dict[str, object] = {}
        for name, (res, args) in _NATIVES.items():
            f = getattr(L, PREFIX + name)
            f.restype = res
            f.argtypes = [c_void_p, c_void_p] + args
            self.fn[name] = f

    # -- JVM objects --------------------------------------------------------
    def string(self, s: Optional[str]):
        return self.L.fj_string(s.encode()) if s is not None else None

    def doubles(self, v) -> int:
        a = np.ascontiguousarray(v, np.float64)
        return self.L.fj_doubles(a.ctypes.data_as(c_void_p), a.shape[0])

    def read(self, o):
        """A Java value as Python: str, numpy array, or None."""
        if not o:
            return None
        k, n = self.L.fj_kind(o), self.L.fj_len(o)
        if k == FJ_STRING:
            return self.L.fj_name(o).decode()
        dt = {FJ_BYTES: np.int8, FJ_INTS: np.int32, FJ_DOUBLES: np.float64}[k]
        if n == 0:
            return np.zeros(0, dt)
        return np.ctypeslib.as_array(ctypes.cast(self.L.fj_data(o), POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                     (n,)).copy()

    def field(self, o, name: str):
        return self.read(self.L.fj_field(o, name.encode()))

    def class_name(self, o) -> str:
        return self.L.fj_name(o).decode()

    def take_exception(self):
        cls, msg = ctypes.create_string_buffer(256), ctypes.create_string_buffer(4096)
        if self.L.fj_take_exception(cls, 256, msg, 4096):
            return cls.value.decode(), msg.value.decode()
        return None

    def violations(self) -> int:
        return self.L.fj_violations()

    def utf_outstanding(self) -> int:
        return self.L.fj_utf_outstanding()

    def fail_alloc_at(self, k: int) -> None:
        self.L.fj_fail_alloc_at(k)

    def reset(self) -> None:
        self.L.fj_reset()

    def call(self, name: str, *args):
        """One native call; a pending exception is raised as JavaException."""
        r = self.fn[name](self.env, None, *args)
        exc = self.take_exception()
        if exc:
            raise JavaException(*exc)
        return r


class JniStore:
    """DBIndexStoreHip's native half, driven through the fake JVM."""

    def __init__(self, jvm: Jvm, cparams, device: int = 0, mandatory: Optional[str] = None):
        self.j = jvm
        p = cparams
        cleave = "".join(chr(c) for c in range(256) if p.cleave[c])
        nocut = "".join(chr(c) for c in range(256) if p.nocut[c])
        self.h = jvm.call("create", jvm.doubles(np.array(p.mass[:], np.float64)), jvm.string(cleave),
                          jvm.string(nocut), jvm.string(mandatory), p.max_missed, p.semi, p.min_mh, p.max_mh,
                          p.add_h2o_proton, p.h2o_proton, p.cterm, p.nterm, p.mass_group_factor,
                          p.index_factor, device)

    def close(self) -> None:
        if self.h:
            self.j.call("close0", self.h)
            self.h = 0

    def __getattr__(self, name):
        if name + "0" in _NATIVES:
            j = self.j
            conv = {str: j.string}

            def f(*args):
                out = [conv.get(type(a), lambda x: x)(a) for a in args]
                return j.call(name + "0", self.h, *out)
            return f
        raise AttributeError(name)

    def ranges(self, native: str, masses, tols):
        return self.j.call(native, self.h, self.j.doubles(masses), self.j.doubles(tols))

    def seq_list(self, o) -> List[tuple]:
        """SeqList (DBIndexStoreHip.java:38-50) -> (sequence, mass, protein ids,
        left, right, offset, length) per IndexedSequence, as toList builds them
        without a ProteinCache."""
        j = self.j
        assert j.class_name(o) == "edu/scripps/yates/dbindex/hip/DBIndexStoreHip$SeqList"
        mass, so, chars = j.field(o, "mass"), j.field(o, "seqOff"), j.field(o, "seqChars")
        left, right = j.field(o, "left"), j.field(o, "right")
        po, pids, poff = j.field(o, "protOff"), j.field(o, "protIds"), j.field(o, "pepOff")
        txt = chars.tobytes().decode("latin-1")
        lt, rt = left.tobytes().decode("latin-1"), right.tobytes().decode("latin-1")
        out = []
        for i in range(mass.shape[0]):
            out.append((txt[so[i]:so[i + 1]], float(mass[i]), [int(x) for x in pids[po[i]:po[i + 1]]],
                        lt[3 * i:3 * i + 3], rt[3 * i:3 * i + 3], int(poff[i]), int(so[i + 1] - so[i])))
        return out
