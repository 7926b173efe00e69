"""Batch engine: the device-resident peptide index behind the C-ABI
(``dbi_open`` / ``dbi_build*`` / ``dbi_query*`` / ``dbi_peptides`` ...).

Inputs are numpy arrays (copied to HBM) or device pointers (``build_device`` /
``query_device``, e.g. from ``torch.Tensor.data_ptr()`` on a ROCm tensor), so
the timed path can start with residues already resident in HBM.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from . import _native
from ._native import DbiDeviceHits, DbiDeviceIndex, DbiQueryResult, DbiStats, check
from .fasta import PackedProteins
from .params import DBIndexSearchParams, DbiParams


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class BuildStats:
    n_residues: int
    n_proteins: int
    n_total: int      # totalSeqCount: peptides indexed (incl. bucket-dropped)
    n_dropped: int
    n_kept: int
    n_unique: int
    n_keys: int       # getNumberSequences(): distinct mass-key rows
    n_bins: int
    n_big_bins: int
    device_bytes: int
    build_ms: float
    digest_ms: float


class Engine:
    def __init__(self, params, device: int = 0, options=None):
        """options: {name: value} for dbi_set_option / dbi_set_option_str
        (tuning switches and test hooks, e.g. {"depth_bins": 0})."""
        if isinstance(params, DBIndexSearchParams):
            params = params.to_c()
        assert isinstance(params, DbiParams)
        self.cparams = params
        self.device = device
        h = ctypes.c_void_p()
        check(_native.lib().dbi_open(ctypes.byref(params), device, ctypes.byref(h)))
        self.h = h
        self._keep = None
        for k, v in (options or {}).items():
            self.set_option(k, v)

    def set_option(self, name: str, value) -> None:
        """dbi_set_option (int) or dbi_set_option_str (str)."""
        if isinstance(value, str):
            check(_native.lib().dbi_set_option_str(self.h, name.encode(), value.encode()))
        else:
            check(_native.lib().dbi_set_option(self.h, name.encode(), int(value)))

    def close(self) -> None:
        if getattr(self, "h", None):
            _native.lib().dbi_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- build ---------------------------------------------------------------
    def build(self, proteins: PackedProteins) -> BuildStats:
        res = np.ascontiguousarray(proteins.residues, dtype=np.uint8)
        off = np.ascontiguousarray(proteins.offsets, dtype=np.uint64)
        check(_native.lib().dbi_build(self.h, _p(res), res.shape[0], _p(off), off.shape[0] - 1))
        return self.stats()

    def build_fasta(self, path: str, threads: int = 0, with_defs: bool = False):
        """The one-off build from a FASTA file in one call (dbi_build_fasta,
        DBIndexer.run).  Returns (BuildStats, offsets, defs): the file's
        protein offsets (u64, P+1) and, with_defs, its definitions."""
        out = ctypes.POINTER(_native.DbiFasta)()
        check(_native.lib().dbi_build_fasta(self.h, path.encode(), threads, ctypes.byref(out)))
        try:
            f = out.contents
            P = int(f.n_proteins)
            offs = np.ctypeslib.as_array(f.offsets, shape=(P + 1,)).astype(np.uint64)
            defs = []
            if with_defs and P:
                doff = np.ctypeslib.as_array(f.def_off, shape=(P + 1,))
                raw = ctypes.string_at(f.defs, int(doff[-1])).decode("latin-1")
                defs = [raw[int(doff[i]):int(doff[i + 1])] for i in range(P)]
        finally:
            _native.lib().dbi_fasta_free(out)
        return self.stats(), offs, defs

    def build_device(self, d_residues: int, n_res: int, d_offsets: int, n_prot: int,
                     stream: int = 0) -> BuildStats:
        check(_native.lib().dbi_build_device(self.h, ctypes.c_void_p(d_residues), n_res,
                                             ctypes.c_void_p(d_offsets), n_prot,
                                             ctypes.c_void_p(stream) if stream else None))
        return self.stats()

    def build_occurrences(self, proteins: PackedProteins, mass, prot_id, offset, length,
                          n_dropped_extra: int = 0) -> BuildStats:
        res = np.ascontiguousarray(proteins.residues, dtype=np.uint8)
        off = np.ascontiguousarray(proteins.offsets, dtype=np.uint64)
        m = np.ascontiguousarray(mass, np.float64)
        pid = np.ascontiguousarray(prot_id, np.uint32)
        o = np.ascontiguousarray(offset, np.uint32)
        ln = np.ascontiguousarray(length, np.uint32)
        check(_native.lib().dbi_build_occurrences(self.h, _p(res), res.shape[0], _p(off), off.shape[0] - 1,
                                                  _p(m), _p(pid), _p(o), _p(ln), m.shape[0], n_dropped_extra))
        return self.stats()

    def synth_proteome(self, seed: int, p_begin: int, n_prot: int, res_base: int, tables):
        """Proteins [p_begin, p_begin+n_prot) of the counter-based synthetic
        proteome, generated in HBM (dbi_synth_proteome): (d_res, d_off, n_res),
        device pointers owned by this engine until its next call."""
        lt = np.ascontiguousarray(tables[0], np.uint16)
        rt = np.ascontiguousarray(tables[1], np.uint8)
        assert lt.shape == (4096,) and rt.shape == (65536,)
        d_res, d_off, n_res = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        check(_native.lib().dbi_synth_proteome(self.h, seed, p_begin, n_prot, res_base, _p(lt), _p(rt),
                                               ctypes.byref(d_res), ctypes.byref(d_off), ctypes.byref(n_res)))
        return d_res.value or 0, d_off.value or 0, n_res.value

    def count_device(self, d_residues: int, n_res: int, d_offsets: int, n_prot: int) -> Tuple[int, int]:
        """COUNT-mode digest (dbi_count): (totalSeqCount, bucket drops)."""
        t, d = ctypes.c_uint64(), ctypes.c_uint64()
        check(_native.lib().dbi_count(self.h, ctypes.c_void_p(d_residues), n_res, ctypes.c_void_p(d_offsets),
                                      n_prot, ctypes.byref(t), ctypes.byref(d)))
        return t.value, d.value

    def count_buckets_device(self, d_residues: int, n_res: int, d_offsets: int, n_prot: int,
                             d_bucket_counts: int) -> Tuple[int, int]:
        """COUNT-mode digest with the SQLiteMult bucket of every occurrence
        (dbi_count_buckets): adds into the device array d_bucket_counts
        (index_factor + 1 u64); returns (totalSeqCount, bucket drops)."""
        t, d = ctypes.c_uint64(), ctypes.c_uint64()
        check(_native.lib().dbi_count_buckets(self.h, ctypes.c_void_p(d_residues), n_res, ctypes.c_void_p(d_offsets),
                                              n_prot, ctypes.c_void_p(d_bucket_counts), ctypes.byref(t),
                                              ctypes.byref(d)))
        return t.value, d.value

    def save(self, path: str) -> None:
        """The built index + its proteome to one file (dbi_index_save)."""
        check(_native.lib().dbi_index_save(self.h, path.encode()))

    def load(self, path: str) -> BuildStats:
        """Replace this engine's index by a saved one (same parameters only)."""
        check(_native.lib().dbi_index_load(self.h, path.encode()))
        return self.stats()

    def stats(self) -> BuildStats:
        st = DbiStats()
        check(_native.lib().dbi_stats_get(self.h, ctypes.byref(st)))
        return BuildStats(*[getattr(st, f) for f, _ in DbiStats._fields_])

    # -- queries -------------------------------------------------------------
    def query(self, mass, tol) -> Tuple[np.ndarray, np.ndarray]:
        """(first, count) per query: ids first..first+count-1 of the mass-sorted
        unique table (getSequences(m, tol) semantics)."""
        m = np.ascontiguousarray(np.atleast_1d(mass), np.float64)
        t = np.ascontiguousarray(np.broadcast_to(np.atleast_1d(tol), m.shape), np.float64)
        first = np.zeros(m.shape[0], np.uint64)
        count = np.zeros(m.shape[0], np.uint64)
        check(_native.lib().dbi_query(self.h, _p(m), _p(t), m.shape[0], _p(first), _p(count)))
        return first, count

    def query_device(self, d_mass: int, d_tol: int, nq: int, d_first: int, d_count: int,
                     stream: int = 0) -> None:
        check(_native.lib().dbi_query_device(self.h, ctypes.c_void_p(d_mass), ctypes.c_void_p(d_tol), nq,
                                             ctypes.c_void_p(d_first), ctypes.c_void_p(d_count),
                                             ctypes.c_void_p(stream) if stream else None))

    def query_prepare(self) -> None:
        """Builds the query directory of the current index now (dbi_query_prepare)."""
        check(_native.lib().dbi_query_prepare(self.h))

    def query_hits_device(self, d_mass: int, d_tol: int, nq: int) -> DbiDeviceHits:
        """Materialised hits in HBM (dbi_query_hits_device): per query its unique
        ids and their protein ids; device pointers owned by the engine."""
        out = DbiDeviceHits()
        check(_native.lib().dbi_query_hits_device(self.h, ctypes.c_void_p(d_mass), ctypes.c_void_p(d_tol), nq,
                                                  ctypes.byref(out)))
        return out

    def query_hits(self, mass, tol):
        """Host copy of query_hits_device for numpy inputs: dict(row, ids, occ_row,
        hit_occ, prot)."""
        m = np.ascontiguousarray(np.atleast_1d(mass), np.float64)
        t = np.ascontiguousarray(np.broadcast_to(np.atleast_1d(tol), m.shape), np.float64)
        dm, dt = _native.DeviceBuffer.from_numpy(m, self.device), _native.DeviceBuffer.from_numpy(t, self.device)
        r = self.query_hits_device(dm.ptr, dt.ptr, m.shape[0])
        out = {}
        for name, ptr, dt_, n in (("row", r.row, np.uint64, r.nq + 1), ("ids", r.ids, np.uint32, r.n_hits),
                                  ("occ_row", r.occ_row, np.uint64, r.nq + 1),
                                  ("hit_occ", r.hit_occ, np.uint32, r.n_hits),
                                  ("prot", r.prot, np.uint32, r.n_prot_ids)):
            a = np.zeros(n, dt_)
            if n:
                check(_native.lib().dbi_dev_copy_d2h(self.device, a.ctypes.data_as(ctypes.c_void_p),
                                                     ctypes.c_void_p(ptr), a.nbytes))
            out[name] = a
        return out

    def query_csr(self, mass, tol) -> Tuple[np.ndarray, np.ndarray]:
        m = np.ascontiguousarray(np.atleast_1d(mass), np.float64)
        t = np.ascontiguousarray(np.broadcast_to(np.atleast_1d(tol), m.shape), np.float64)
        r = ctypes.POINTER(DbiQueryResult)()
        check(_native.lib().dbi_query_csr(self.h, _p(m), _p(t), m.shape[0], ctypes.byref(r)))
        try:
            nq, nh = r.contents.nq, r.contents.n_hits
            row = np.ctypeslib.as_array(r.contents.row_ptr, shape=(nq + 1,)).copy()
            ids = np.ctypeslib.as_array(r.contents.ids, shape=(max(nh, 1),))[:nh].copy()
        finally:
            _native.lib().dbi_query_result_free(r)
        return row, ids

    def peptides(self, ids):
        ids = np.ascontiguousarray(np.atleast_1d(ids), np.uint64)
        n = ids.shape[0]
        out = dict(mass=np.zeros(n, np.float64), prot_id=np.zeros(n, np.uint32),
                   offset=np.zeros(n, np.uint32), length=np.zeros(n, np.uint32),
                   occ_begin=np.zeros(n, np.uint64), occ_end=np.zeros(n, np.uint64))
        check(_native.lib().dbi_peptides(self.h, _p(ids), n, _p(out["mass"]), _p(out["prot_id"]),
                                         _p(out["offset"]), _p(out["length"]), _p(out["occ_begin"]),
                                         _p(out["occ_end"])))
        return out

    def occurrences(self, begin: int, end: int) -> np.ndarray:
        out = np.zeros(max(end - begin, 0), np.uint32)
        check(_native.lib().dbi_occurrences(self.h, begin, end, _p(out)))
        return out

    def export(self):
        st = self.stats()
        U, K = st.n_unique, st.n_kept
        out = dict(mass=np.zeros(U, np.float64), prot_id=np.zeros(U, np.uint32),
                   offset=np.zeros(U, np.uint32), length=np.zeros(U, np.uint32),
                   occ_off=np.zeros(U + 1, np.uint64), occ_prot=np.zeros(K, np.uint32))
        check(_native.lib().dbi_export(self.h, _p(out["mass"]), _p(out["prot_id"]), _p(out["offset"]),
                                       _p(out["length"]), _p(out["occ_off"]), _p(out["occ_prot"])))
        return out

    def entry_keys(self) -> np.ndarray:
        n = ctypes.c_uint64()
        check(_native.lib().dbi_entry_keys(self.h, None, 0, ctypes.byref(n)))
        keys = np.zeros(n.value, np.int32)
        check(_native.lib().dbi_entry_keys(self.h, _p(keys), n.value, ctypes.byref(n)))
        return keys

    def set_bucket_drop(self, on: bool) -> None:
        """``dbi_set_bucket_drop``: off = MassRangeFilteringIndex semantics (no buckets)."""
        check(_native.lib().dbi_set_bucket_drop(self.h, 1 if on else 0))

    def set_windows(self, mass=None, tol=None, on: bool = True) -> None:
        """``dbi_set_windows``: the next builds keep only peptides inside a window."""
        m = np.ascontiguousarray(mass if mass is not None else [], np.float64)
        t = np.ascontiguousarray(tol if tol is not None else [], np.float64)
        check(_native.lib().dbi_set_windows(self.h, m.ctypes.data_as(ctypes.c_void_p),
                                            t.ctypes.data_as(ctypes.c_void_p), m.shape[0], 1 if on else 0))

    def rebuild(self) -> BuildStats:
        """``dbi_rebuild``: build again over the resident inputs of the last build."""
        check(_native.lib().dbi_rebuild(self.h))
        return self.stats()

    def set_cold(self) -> None:
        """The next build takes the cold path (count + emit digest, radix tail,
        full list grids) with the device buffers kept (dbi_set_cold)."""
        check(_native.lib().dbi_set_cold(self.h))

    def set_timing(self, on: bool, only: str = "") -> None:
        """Per-kernel HIP events carried by the dispatch packets (default: every
        stage); ``only`` restricts them to the stages of that name."""
        check(_native.lib().dbi_set_timing(self.h, 1 if on else 0, only.encode()))

    def stage_times(self):
        """[(kernel, ms, algorithmic bytes)] of the last build, from the HIP
        events carried by each kernel's dispatch packet (0 ms if untimed)."""
        n = ctypes.c_uint64()
        check(_native.lib().dbi_stage_times(self.h, None, None, None, 0, ctypes.byref(n)))
        k = n.value
        names = (ctypes.c_char_p * max(k, 1))()
        ms = np.zeros(max(k, 1), np.float64)
        by = np.zeros(max(k, 1), np.float64)
        check(_native.lib().dbi_stage_times(self.h, ctypes.cast(names, ctypes.c_void_p), _p(ms), _p(by), k,
                                            ctypes.byref(n)))
        return [(names[i].decode(), float(ms[i]), float(by[i])) for i in range(k)]

    def device_view(self) -> DbiDeviceIndex:
        v = DbiDeviceIndex()
        check(_native.lib().dbi_device_view(self.h, ctypes.byref(v)))
        return v
