"""oracle/cref.py — TEST INFRASTRUCTURE ONLY: ctypes view of oracle/cpu_ref.cpp.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product path (dbindex_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libdbi_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, U8, U32, U64, D = (ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8),
                              ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64),
                              ctypes.POINTER(ctypes.c_double))
        L.oref_digest.argtypes = [P, P, P, ctypes.c_uint64, P, P, P, P, P, ctypes.c_uint64, U64]
        L.oref_build.argtypes = [P, P, P, ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
        L.oref_build_occurrences.argtypes = [P, P, P, ctypes.c_uint64, P, P, P, P,
                                             ctypes.c_uint64, ctypes.POINTER(ctypes.c_void_p)]
        L.oref_free.argtypes = [P]
        for f in ("oref_n_total", "oref_n_dropped", "oref_n_unique", "oref_n_kept", "oref_n_keys"):
            getattr(L, f).argtypes = [P]
            getattr(L, f).restype = ctypes.c_uint64
        L.oref_build_seconds.argtypes = [P]
        L.oref_build_seconds.restype = ctypes.c_double
        L.oref_entry_keys.argtypes = [P, P]
        L.oref_unique.argtypes = [P, P, P, P, P, P, P]
        L.oref_query.argtypes = [P, ctypes.c_double, ctypes.c_double, P, ctypes.c_uint64, U64]
        L.oref_query_ranges.argtypes = [P, P, P, ctypes.c_uint64, P, ctypes.c_uint64, U64]
        L.oref_formula_mass.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
        L.oref_formula_mass.restype = ctypes.c_double
        L.oref_calculate_mass.argtypes = [P, P, ctypes.c_uint64]
        L.oref_calculate_mass.restype = ctypes.c_double
        L.oref_tolerance_in_dalton.argtypes = [ctypes.c_double, ctypes.c_double]
        L.oref_tolerance_in_dalton.restype = ctypes.c_double
        L.oref_set_threads.argtypes = [ctypes.c_int]
        L.oref_count.argtypes = [P, P, P, ctypes.c_uint64, U64, U64]
        L.oref_count_buckets.argtypes = [P, P, P, ctypes.c_uint64, P]
        L.oref_query_batch.argtypes = [P, P, P, ctypes.c_uint64, P, P]
        _lib = L
    return _lib


def set_threads(n: int) -> None:
    """Worker threads of the oracle's build, digest and batched query (1 = the
    reference's single-threaded path; results do not depend on it)."""
    lib().oref_set_threads(int(n))


class threads:
    """Context manager: ``with cref.threads(16): ...``, back to 1 afterwards."""

    def __init__(self, n: int):
        self.n = n

    def __enter__(self):
        set_threads(self.n)
        return self

    def __exit__(self, *exc):
        set_threads(1)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class Digest:
    mass: np.ndarray
    pid: np.ndarray
    offset: np.ndarray
    length: np.ndarray
    dropped: np.ndarray


def digest(cparams, residues: np.ndarray, offsets: np.ndarray) -> Digest:
    L = lib()
    residues = np.ascontiguousarray(residues, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = ctypes.c_uint64()
    P = offsets.shape[0] - 1
    rc = L.oref_digest(ctypes.byref(cparams), _ptr(residues), _ptr(offsets), P,
                       None, None, None, None, None, 0, ctypes.byref(n))
    if rc != 0:  # a protein the reference's cutSeq throws on (inline PTM at its start, '[' without ']')
        raise ValueError(f"oref_digest failed: {rc}")
    k = n.value
    out = Digest(np.zeros(k, np.float64), np.zeros(k, np.uint32), np.zeros(k, np.uint32),
                 np.zeros(k, np.uint32), np.zeros(k, np.uint8))
    if k:
        rc = L.oref_digest(ctypes.byref(cparams), _ptr(residues), _ptr(offsets), P,
                           _ptr(out.mass), _ptr(out.pid), _ptr(out.offset), _ptr(out.length),
                           _ptr(out.dropped), k, ctypes.byref(n))
        assert rc == 0
    return out


def count(cparams, residues: np.ndarray, offsets: np.ndarray):
    """(totalSeqCount, bucket drops) of cutSeq over every protein (oref_count)."""
    residues = np.ascontiguousarray(residues, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    t, d = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().oref_count(ctypes.byref(cparams), _ptr(residues), _ptr(offsets), offsets.shape[0] - 1,
                          ctypes.byref(t), ctypes.byref(d))
    if rc != 0:
        raise ValueError(f"oref_count failed: {rc}")
    return t.value, d.value


def count_buckets(cparams, residues: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    """Occurrences per SQLiteMult bucket ((int)m / BUCKET_MASS_RANGE), the last
    entry = past the last bucket (oref_count_buckets): index_factor + 1 counts."""
    residues = np.ascontiguousarray(residues, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    hist = np.zeros(int(cparams.index_factor) + 1, np.uint64)
    rc = lib().oref_count_buckets(ctypes.byref(cparams), _ptr(residues), _ptr(offsets), offsets.shape[0] - 1,
                                  _ptr(hist))
    if rc != 0:
        raise ValueError(f"oref_count_buckets failed: {rc}")
    return hist


class Index:
    """The oracle's store: buckets -> rows -> merged peptides."""

    def __init__(self, cparams, residues: np.ndarray, offsets: np.ndarray, occurrences=None):
        L = lib()
        self._keep = (np.ascontiguousarray(residues, dtype=np.uint8),
                      np.ascontiguousarray(offsets, dtype=np.uint64))
        self.params = cparams
        h = ctypes.c_void_p()
        P = offsets.shape[0] - 1
        if occurrences is None:
            rc = L.oref_build(ctypes.byref(cparams), _ptr(self._keep[0]), _ptr(self._keep[1]),
                              P, ctypes.byref(h))
        else:
            m, pid, off, ln = (np.ascontiguousarray(occurrences[0], np.float64),
                               np.ascontiguousarray(occurrences[1], np.uint32),
                               np.ascontiguousarray(occurrences[2], np.uint32),
                               np.ascontiguousarray(occurrences[3], np.uint32))
            rc = L.oref_build_occurrences(ctypes.byref(cparams), _ptr(self._keep[0]),
                                          _ptr(self._keep[1]), P, _ptr(m), _ptr(pid), _ptr(off),
                                          _ptr(ln), m.shape[0], ctypes.byref(h))
        if rc != 0:
            raise ValueError(f"oref_build failed: {rc}")
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib().oref_free(self.h)
            self.h = None

    @property
    def build_seconds(self) -> float:
        return lib().oref_build_seconds(self.h)

    @property
    def n_total(self) -> int:
        return lib().oref_n_total(self.h)

    @property
    def n_dropped(self) -> int:
        return lib().oref_n_dropped(self.h)

    @property
    def n_kept(self) -> int:
        return lib().oref_n_kept(self.h)

    @property
    def n_unique(self) -> int:
        return lib().oref_n_unique(self.h)

    @property
    def n_keys(self) -> int:
        return lib().oref_n_keys(self.h)

    def entry_keys(self) -> np.ndarray:
        k = np.zeros(self.n_keys, np.int32)
        lib().oref_entry_keys(self.h, _ptr(k))
        return k

    def unique(self):
        U, K = self.n_unique, self.n_kept
        mass = np.zeros(U, np.float64)
        pid = np.zeros(U, np.uint32)
        off = np.zeros(U, np.uint32)
        ln = np.zeros(U, np.uint32)
        occ_off = np.zeros(U + 1, np.uint64)
        occ_pid = np.zeros(K, np.uint32)
        lib().oref_unique(self.h, _ptr(mass), _ptr(pid), _ptr(off), _ptr(ln), _ptr(occ_off),
                          _ptr(occ_pid))
        return dict(mass=mass, prot_id=pid, offset=off, length=ln, occ_off=occ_off,
                    occ_prot=occ_pid)

    def query(self, mass: float, tol: float) -> np.ndarray:
        L = lib()
        n = ctypes.c_uint64()
        L.oref_query(self.h, mass, tol, None, 0, ctypes.byref(n))
        ids = np.zeros(n.value, np.uint64)
        if n.value:
            L.oref_query(self.h, mass, tol, _ptr(ids), n.value, ctypes.byref(n))
        return ids

    def query_ranges(self, masses, tols) -> np.ndarray:
        L = lib()
        m = np.ascontiguousarray(masses, np.float64)
        t = np.ascontiguousarray(tols, np.float64)
        n = ctypes.c_uint64()
        L.oref_query_ranges(self.h, _ptr(m), _ptr(t), m.shape[0], None, 0, ctypes.byref(n))
        ids = np.zeros(n.value, np.uint64)
        if n.value:
            L.oref_query_ranges(self.h, _ptr(m), _ptr(t), m.shape[0], _ptr(ids), n.value,
                                ctypes.byref(n))
        return ids

    def query_batch(self, masses, tols):
        """(first, count) per query, as the engine reports them (contiguous
        ranges; first = 0 when count = 0), oref_query_batch."""
        m = np.ascontiguousarray(masses, np.float64)
        t = np.ascontiguousarray(tols, np.float64)
        first = np.zeros(m.shape[0], np.uint64)
        count = np.zeros(m.shape[0], np.uint64)
        rc = lib().oref_query_batch(self.h, _ptr(m), _ptr(t), m.shape[0], _ptr(first), _ptr(count))
        assert rc == 0, "non-contiguous oracle result"
        return first, count


def formula_mass(formula: str) -> float:
    """The C++ oracle's FormulaCalculator restatement (NaN: unknown element)."""
    b = formula.encode()
    return lib().oref_formula_mass(b, len(b))


def calculate_mass(cparams, seq: str) -> float:
    b = np.frombuffer(seq.encode("ascii"), dtype=np.uint8).copy()
    return lib().oref_calculate_mass(ctypes.byref(cparams), _ptr(b), b.shape[0])


def tolerance_in_dalton(mass: float, ppm: float) -> float:
    return lib().oref_tolerance_in_dalton(mass, ppm)


def cut_and_search(cparams, residues: np.ndarray, offsets: np.ndarray, masses, tols) -> dict:
    """DBIndexer.cutAndSearch over MassRangeFilteringIndex (DBIndexer.java:707-747,
    MassRangeFilteringIndex.java:40-130) on the C++ digest: the filtering store
    has no buckets and no mandatory-residue filter (so mandatory_count = 0 and
    every occurrence counts, dropped or not), and keeps the peptides with
    min <= m <= max for some range.  SKIP_PROTEIN_START only ends a start's walk
    once m exceeds every range, after which masses never fall back in range
    (residue masses >= 0), so filtering the full digest gives the same set --
    tests/test_oracle.py pins this against pyref.cut_and_search, which runs the
    filter inside the walk.  Same return form as pyref.cut_and_search."""
    cp = type(cparams)()
    ctypes.memmove(ctypes.byref(cp), ctypes.byref(cparams), ctypes.sizeof(cparams))
    cp.mandatory_count = 0
    d = digest(cp, residues, offsets)
    lo = np.asarray(masses, np.float64) - np.asarray(tols, np.float64)
    hi = np.asarray(masses, np.float64) + np.asarray(tols, np.float64)
    keep = np.zeros(d.mass.shape[0], bool)
    for a, b in zip(lo, hi):  # NaN bounds select nothing
        keep |= (d.mass >= a) & (d.mass <= b)
    res = np.asarray(residues, np.uint8).tobytes()
    offs = np.asarray(offsets, np.uint64)
    out: dict = {}
    for i in np.nonzero(keep)[0]:
        pid, off, ln = int(d.pid[i]), int(d.offset[i]), int(d.length[i])
        p0, p1 = int(offs[pid]), int(offs[pid + 1])
        seq = res[p0 + off: p0 + off + ln].decode("ascii")
        e = out.get(seq)
        if e is None:
            prot = res[p0:p1].decode("ascii")
            end = off + ln - 1
            left = prot[max(0, off - 3): off].rjust(3, "-")
            right = prot[end + 1: end + 1 + max(0, min(3, len(prot) - end - 1))].ljust(3, "-")
            out[seq] = (float(d.mass[i]), off, ln, left, right, [pid])
        elif pid not in e[5]:
            e[5].append(pid)
    return out
