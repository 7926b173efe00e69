"""ctypes binding of the C-ABI in include/dbindex_hip.h (libdbindex_hip.so).

This is the Python twin of the JNI shim described in INTEGRATION.md: every
symbol is bound with its exact C signature.  There is no fallback path — if
the in-tree HIP library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

from .params import DbiParams

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DBI_LIB_PATH") or os.path.join(HERE, "libdbindex_hip.so")  # override: experiments
# the test-hook variant (options test_fail / test_split_skew; dbindex_amd/build.py):
# only the failure-injection tests load it, in processes of their own (DBI_LIB_PATH)
HOOKS_PATH = os.path.join(HERE, "libdbindex_hip_hooks.so")

DBI_OK, DBI_E_INVALID, DBI_E_OOM, DBI_E_HIP, DBI_E_RCCL, DBI_E_STATE = 0, -1, -2, -3, -4, -5
FILTER_INCLUDE, FILTER_SKIP, FILTER_SKIP_PROTEIN_START = 0, 1, 2
ERROR_NAMES = {-1: "DBI_E_INVALID", -2: "DBI_E_OOM", -3: "DBI_E_HIP", -4: "DBI_E_RCCL", -5: "DBI_E_STATE"}


class DBIndexStoreException(Exception):
    """Mirror of edu.scripps.yates.utilities.fasta.dbindex.DBIndexStoreException:
    every non-zero status of the C-ABI is raised, never swallowed."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


class DbiStats(ctypes.Structure):
    _fields_ = [
        ("n_residues", c_uint64), ("n_proteins", c_uint64), ("n_total", c_uint64),
        ("n_dropped", c_uint64), ("n_kept", c_uint64), ("n_unique", c_uint64),
        ("n_keys", c_uint64), ("n_bins", c_uint64), ("n_big_bins", c_uint64),
        ("device_bytes", c_uint64), ("build_ms", c_double), ("digest_ms", c_double),
    ]


class DbiShardStats(ctypes.Structure):
    _fields_ = [
        ("rank", c_int32), ("nshards", c_int32), ("p_begin", c_uint64), ("p_end", c_uint64),
        ("key_lo", c_int32), ("key_hi", c_int32), ("n_total", c_uint64), ("n_dropped", c_uint64),
        ("n_sent", c_uint64), ("n_received", c_uint64), ("n_unique", c_uint64), ("n_keys", c_uint64),
        ("g_total", c_uint64), ("g_dropped", c_uint64), ("g_kept", c_uint64), ("g_unique", c_uint64),
        ("g_keys", c_uint64), ("digest_ms", c_double), ("partition_ms", c_double),
        ("exchange_ms", c_double), ("merge_ms", c_double), ("merge_gpu_ms", c_double),
        ("split_sampled", c_int32), ("split_rounds", c_int32), ("split_held", c_int32), ("reserved0", c_int32),
    ]


SHARD_SAMPLES = 4096  # DBI_SHARD_SAMPLES
MAX_SHARDS = 64       # DBI_MAX_SHARDS


class DbiFasta(ctypes.Structure):
    _fields_ = [("n_proteins", c_uint64), ("n_residues", c_uint64), ("residues", c_void_p),
                ("offsets", POINTER(c_uint64)), ("defs", c_void_p), ("def_off", POINTER(c_uint64)),
                ("n_uniprot", c_uint64)]


class DbiQueryResult(ctypes.Structure):
    _fields_ = [("nq", c_uint64), ("n_hits", c_uint64), ("row_ptr", POINTER(c_uint64)),
                ("ids", POINTER(c_uint64))]


class DbiDeviceIndex(ctypes.Structure):
    _fields_ = [("mass", c_void_p), ("prot_id", c_void_p), ("offset", c_void_p), ("length", c_void_p),
                ("occ_off", c_void_p), ("occ_prot", c_void_p), ("n_unique", c_uint64),
                ("n_kept", c_uint64)]


class DbiDeviceHits(ctypes.Structure):
    _fields_ = [("row", c_void_p), ("ids", c_void_p), ("occ_row", c_void_p), ("hit_occ", c_void_p),
                ("prot", c_void_p), ("nq", c_uint64), ("n_hits", c_uint64), ("n_prot_ids", c_uint64)]


class DbiRuntimeInfo(ctypes.Structure):
    _fields_ = [("hip_runtime_version", c_int), ("hip_driver_version", c_int), ("rccl_version", c_int),
                ("libamdhip64", ctypes.c_char * 512), ("librccl", ctypes.c_char * 512)]


class DbiSeqList(ctypes.Structure):
    _fields_ = [
        ("n", c_uint64), ("mass", POINTER(c_double)), ("seq_off", POINTER(c_uint64)),
        ("seq_chars", c_void_p), ("res_left", c_void_p), ("res_right", c_void_p),
        ("prot_off", POINTER(c_uint64)), ("prot_ids", POINTER(c_uint32)),
        ("offset", POINTER(c_uint32)), ("length", POINTER(c_uint32)), ("unique_id", POINTER(c_uint64)),
    ]


# (name, restype, argtypes) for every exported symbol of include/dbindex_hip.h
P = c_void_p
SIGNATURES = [
    ("dbi_params_default", None, [POINTER(DbiParams), c_int32, c_int32]),
    ("dbi_open", c_int, [POINTER(DbiParams), c_int, POINTER(c_void_p)]),
    ("dbi_close", None, [P]),
    ("dbi_build", c_int, [P, P, c_uint64, P, c_uint64]),
    ("dbi_build_device", c_int, [P, P, c_uint64, P, c_uint64, P]),
    ("dbi_build_occurrences", c_int, [P, P, c_uint64, P, c_uint64, P, P, P, P, c_uint64, c_uint64]),
    ("dbi_stats_get", c_int, [P, POINTER(DbiStats)]),
    ("dbi_query", c_int, [P, P, P, c_uint64, P, P]),
    ("dbi_query_device", c_int, [P, P, P, c_uint64, P, P, P]),
    ("dbi_query_csr", c_int, [P, P, P, c_uint64, POINTER(POINTER(DbiQueryResult))]),
    ("dbi_query_result_free", None, [POINTER(DbiQueryResult)]),
    ("dbi_query_prepare", c_int, [P]),
    ("dbi_query_hits_device", c_int, [P, P, P, c_uint64, POINTER(DbiDeviceHits)]),
    ("dbi_peptides", c_int, [P, P, c_uint64, P, P, P, P, P, P]),
    ("dbi_occurrences", c_int, [P, c_uint64, c_uint64, P]),
    ("dbi_export", c_int, [P, P, P, P, P, P, P]),
    ("dbi_entry_keys", c_int, [P, P, c_uint64, POINTER(c_uint64)]),
    ("dbi_device_view", c_int, [P, POINTER(DbiDeviceIndex)]),
    ("dbi_set_timing", c_int, [P, c_int, c_char_p]),
    ("dbi_set_cold", c_int, [P]),
    ("dbi_set_option", c_int, [P, c_char_p, ctypes.c_int64]),
    ("dbi_set_option_str", c_int, [P, c_char_p, c_char_p]),
    ("dbi_set_bucket_drop", c_int, [P, c_int]),
    ("dbi_set_windows", c_int, [P, P, P, c_uint64, c_int]),
    ("dbi_rebuild", c_int, [P]),
    ("dbi_stage_times", c_int, [P, P, P, P, c_uint64, POINTER(c_uint64)]),
    ("dbi_shard_digest", c_int, [P, P, c_uint64, P, c_uint64, c_uint64, c_uint64, c_int, c_int]),
    ("dbi_shard_samples", c_int, [P, P]),
    ("dbi_shard_splitters", c_int, [P, c_int, c_int32, P]),
    ("dbi_shard_splitters_cost", c_int, [P, c_int, c_int32, c_int, P, P, P]),
    ("dbi_shard_cost_update", c_int, [P, c_int, P, P, P]),
    ("dbi_shard_splitters_profiled", c_int, [P, P, c_int, P]),
    ("dbi_shard_partition", c_int, [P, P, P]),
    ("dbi_shard_exchange_local", c_int, [P, c_int]),
    ("dbi_shard_merge", c_int, [P]),
    ("dbi_shard_stats_get", c_int, [P, POINTER(DbiShardStats)]),
    ("dbi_query_sharded", c_int, [P, P, P, P, c_uint64, P, P]),
    ("dbi_query_sharded_local", c_int, [P, c_int, P, P, P, P, P]),
    ("dbi_shard_replicate", c_int, [P, P]),
    ("dbi_shard_replicate_local", c_int, [P, c_int]),
    ("dbi_synth_proteome", c_int, [P, c_uint64, c_uint64, c_uint64, c_uint64, P, P, POINTER(c_void_p),
                                   POINTER(c_void_p), POINTER(c_uint64)]),
    ("dbi_count", c_int, [P, P, c_uint64, P, c_uint64, POINTER(c_uint64), POINTER(c_uint64)]),
    ("dbi_count_buckets", c_int, [P, P, c_uint64, P, c_uint64, P, POINTER(c_uint64), POINTER(c_uint64)]),
    ("dbi_comm_unique_id", c_int, [P]),
    ("dbi_comm_init", c_int, [P, c_int, c_int, c_int, POINTER(c_void_p)]),
    ("dbi_comm_init_host", c_int, [c_char_p, c_int, c_int, c_int, c_uint64, POINTER(c_void_p)]),
    ("dbi_comm_destroy", None, [P]),
    ("dbi_comm_allgatherv", c_int, [P, P, P, P, P]),
    ("dbi_comm_allreduce_f64", c_int, [P, P, P, c_uint32, c_int]),
    ("dbi_comm_allreduce_u64", c_int, [P, P, P, c_uint64, P]),
    ("dbi_runtime_info_get", c_int, [POINTER(DbiRuntimeInfo)]),
    ("dbi_build_sharded", c_int, [P, P, P, c_uint64, P, c_uint64, c_uint64, c_uint64]),
    ("dbi_store_create", c_int, [POINTER(DbiParams), c_int, POINTER(c_void_p)]),
    ("dbi_store_close", None, [P]),
    ("dbi_store_set_device_digest", c_int, [P, c_int]),
    ("dbi_store_init", c_int, [P, c_char_p]),
    ("dbi_store_start_add_seq", c_int, [P]),
    ("dbi_store_stop_add_seq", c_int, [P]),
    ("dbi_store_index_exists", c_int, [P, POINTER(c_int)]),
    ("dbi_store_add_protein_def", c_int, [P, c_int64, c_char_p, c_char_p, c_uint64, POINTER(c_int64)]),
    ("dbi_store_filter_sequence", c_int, [P, c_double, c_char_p, c_uint64, POINTER(c_int)]),
    ("dbi_store_add_sequence", c_int, [P, c_double, c_int32, c_int32, c_int64]),
    ("dbi_store_get_number_sequences", c_int, [P, POINTER(c_int64)]),
    ("dbi_store_get_total_seq_count", c_int, [P, POINTER(c_int64)]),
    ("dbi_store_get_entry_keys", c_int, [P, P, c_uint64, POINTER(c_uint64)]),
    ("dbi_store_engine", c_void_p, [P]),
    ("dbi_store_get_sequences", c_int, [P, c_double, c_double, POINTER(POINTER(DbiSeqList))]),
    ("dbi_store_get_sequences_ranges", c_int, [P, P, P, c_uint64, POINTER(POINTER(DbiSeqList))]),
    ("dbi_store_cut_and_search", c_int, [P, P, P, c_uint64, POINTER(POINTER(DbiSeqList))]),
    ("dbi_seq_list_free", None, [POINTER(DbiSeqList)]),
    ("dbi_store_protein_count", c_int, [P, POINTER(c_uint64)]),
    ("dbi_store_protein_def", c_int, [P, c_uint64, POINTER(c_char_p), POINTER(c_uint64)]),
    ("dbi_store_protein_sequence", c_int, [P, c_uint64, POINTER(c_void_p), POINTER(c_uint64)]),
    ("dbi_index_save", c_int, [P, c_char_p]),
    ("dbi_index_load", c_int, [P, c_char_p]),
    ("dbi_index_file_matches", c_int, [POINTER(DbiParams), c_char_p, POINTER(c_int)]),
    ("dbi_store_set_persist", c_int, [P, c_int]),
    ("dbi_store_set_unindexed", c_int, [P, c_int]),
    ("dbi_fasta_parse", c_int, [P, c_uint64, c_int, POINTER(POINTER(DbiFasta))]),
    ("dbi_fasta_read", c_int, [c_char_p, c_int, POINTER(POINTER(DbiFasta))]),
    ("dbi_fasta_free", None, [POINTER(DbiFasta)]),
    ("dbi_build_fasta", c_int, [P, c_char_p, c_int, POINTER(POINTER(DbiFasta))]),
    ("dbi_dev_alloc", c_int, [c_int, c_uint64, POINTER(c_void_p)]),
    ("dbi_dev_free", c_int, [c_int, P]),
    ("dbi_dev_copy_h2d", c_int, [c_int, P, P, c_uint64]),
    ("dbi_dev_copy_d2h", c_int, [c_int, P, P, c_uint64]),
    ("dbi_dev_copy_d2d", c_int, [c_int, P, P, c_uint64]),
    ("dbi_hbm_copy_bandwidth", c_int, [c_int, c_uint64, c_int, POINTER(c_double)]),
    ("dbi_dev_synchronize", c_int, [c_int]),
    ("dbi_last_error", c_char_p, []),
    ("dbi_abi_version", c_int, []),
    ("dbi_device_count", c_int, [POINTER(c_int)]),
]

_lib = None


def lib():
    """Loads the in-tree HIP library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -m dbindex_amd.build` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        check_single_runtime()
    return _lib


def mapped_runtimes() -> dict:
    """Distinct files of the HIP runtime and of RCCL mapped into this process
    (/proc/self/maps): {"libamdhip64": [...], "librccl": [...]}."""
    found = {"libamdhip64": set(), "librccl": set()}
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                parts = line.split(None, 5)
                if len(parts) < 6:
                    continue
                path = parts[5].strip()
                base = os.path.basename(path)
                for key in found:
                    if base.startswith(key + ".") or base.startswith(key + "-"):
                        found[key].add(os.path.realpath(path))
    except OSError:
        pass
    return {k: sorted(v) for k, v in found.items()}


def check_single_runtime() -> dict:
    """Raises when two HIP runtimes or two RCCLs are mapped into this process
    (e.g. PyTorch's bundled copies next to /opt/rocm's): kernels, device
    memory and communicators of one must never meet the other."""
    m = mapped_runtimes()
    for key, paths in m.items():
        if len(paths) > 1:
            raise ImportError(f"two {key} copies mapped into this process: {paths}; load dbindex_amd before "
                              "anything that brings its own ROCm runtime (torch), or run without it")
    return m


def runtime_info() -> dict:
    """The HIP runtime and RCCL the library is bound to (versions, providing files)."""
    ri = DbiRuntimeInfo()
    check(lib().dbi_runtime_info_get(ctypes.byref(ri)))
    v = ri.rccl_version
    return dict(hip_runtime_version=ri.hip_runtime_version, hip_driver_version=ri.hip_driver_version,
                rccl_version=f"{v // 10000}.{v // 100 % 100}.{v % 100}" if v else None,
                libamdhip64=ri.libamdhip64.decode(errors="replace"), librccl=ri.librccl.decode(errors="replace"),
                mapped=check_single_runtime())


def last_error() -> str:
    m = lib().dbi_last_error()
    return m.decode(errors="replace") if m else ""


def check(rc: int) -> None:
    if rc != 0:
        raise DBIndexStoreException(rc, last_error())


def default_params(max_missed: int = 2, semi: bool = False) -> DbiParams:
    p = DbiParams()
    lib().dbi_params_default(ctypes.byref(p), max_missed, 1 if semi else 0)
    return p


def device_count() -> int:
    n = c_int(0)
    lib().dbi_device_count(ctypes.byref(n))
    return n.value


class DeviceBuffer:
    """HBM allocation owned through the engine's own HIP runtime.

    (PyTorch-ROCm ships a separate libamdhip64; mixing two HIP runtimes in one
    process is order-dependent, so device-resident inputs for the engine are
    allocated here rather than as torch tensors.)"""

    def __init__(self, nbytes: int, device: int = 0):
        self.device = device
        self.nbytes = int(nbytes)
        p = c_void_p()
        check(lib().dbi_dev_alloc(device, self.nbytes, ctypes.byref(p)))
        self.ptr = p.value or 0

    @classmethod
    def from_numpy(cls, a, device: int = 0) -> "DeviceBuffer":
        import numpy as np
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes, device)
        b.upload(a)
        return b

    def upload(self, a) -> None:
        import numpy as np
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        check(lib().dbi_dev_copy_h2d(self.device, c_void_p(self.ptr), a.ctypes.data_as(c_void_p), a.nbytes))

    def download(self, dtype, count: int):
        import numpy as np
        out = np.empty(count, dtype=dtype)
        assert out.nbytes <= self.nbytes
        check(lib().dbi_dev_copy_d2h(self.device, out.ctypes.data_as(c_void_p), c_void_p(self.ptr), out.nbytes))
        return out

    def copy_from_device(self, offset: int, src_ptr: int, nbytes: int) -> None:
        assert offset + nbytes <= self.nbytes
        check(lib().dbi_dev_copy_d2d(self.device, c_void_p(self.ptr + offset), c_void_p(src_ptr), nbytes))

    def free(self) -> None:
        if self.ptr:
            lib().dbi_dev_free(self.device, c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def synchronize(device: int = 0) -> None:
    check(lib().dbi_dev_synchronize(device))
