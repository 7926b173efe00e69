"""Sharded build: one peptide index over the proteins of several GPUs.

Host side of the C-ABI's ``dbi_shard_*`` / ``dbi_comm_*`` / ``dbi_build_sharded``
(include/dbindex_hip.h).  The reference indexes the whole FASTA in one thread
(``DBIndexer.run``, DBIndexer.java:508-684); here every shard digests a
contiguous protein range, records are routed to the shard owning their mass key
``(int)(mass*factor)`` (DBIndexStoreSQLiteByte.java:187), and each owner merges
its key range (IndexMerge.getMergedData, DBIndexStoreSQLiteByteIndexMerge.java:620-719).
Concatenating the owners' unique tables in shard order gives the index of the
whole proteome, identical row for row to a single-device build.

* ``ShardComm`` — an RCCL communicator (one process per GPU); the 128-byte id
  travels through any out-of-band channel (``torch.distributed`` gloo here).
* ``build_sharded_local`` — every shard's handle in one process, exchange by
  device copies (tests; the same phases the RCCL driver runs).
* ``replicate`` / ``replicate_local`` — the owners' slices all-gathered onto
  every rank (north_star's all-gatherv): each handle then holds the whole
  index and answers queries locally.
* ``protein_ranges`` / ``owner_of`` / ``concat_exports`` — host logic shared by
  both drivers and the CPU tests.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _native
from ._native import DbiShardStats, MAX_SHARDS, SHARD_SAMPLES, check
from .engine import Engine

SPLIT_HOLD = 1.10  # owners this balanced (slowest / mean merge time) keep their split (dbi_shard.hip)


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def protein_ranges(offsets: np.ndarray, nshards: int) -> List[Tuple[int, int]]:
    """Contiguous protein ranges balanced by residue count:
    shard r gets proteins [b_r, b_{r+1}) with b_r the first protein whose start
    offset reaches r/n of the residues."""
    off = np.asarray(offsets, dtype=np.uint64)
    P = off.shape[0] - 1
    R = int(off[-1]) if P >= 0 else 0
    bounds = [0]
    for r in range(1, nshards):
        target = (R * r) // nshards
        bounds.append(max(bounds[-1], int(np.searchsorted(off[:P], target, side="left")) if P else 0))
    bounds.append(P)
    return [(bounds[r], bounds[r + 1]) for r in range(nshards)]


def splitters(samples: np.ndarray, nshards: int, factor: int, profile=None) -> np.ndarray:
    """Owner key splitters from every shard's samples (dbi_shard_splitters, host
    only): ``samples`` = nshards blocks of SHARD_SAMPLES masses + 1 weight.
    ``profile`` = (band_split, band_cost): balance records x the cost per
    record of their key band instead of records (dbi_shard_splitters_cost)."""
    s = np.ascontiguousarray(samples, np.float64).reshape(nshards * (SHARD_SAMPLES + 1))
    out = np.zeros(max(nshards - 1, 1), np.int32)
    if profile is None:
        check(_native.lib().dbi_shard_splitters(_p(s), nshards, factor, _p(out)))
    else:
        bc = np.ascontiguousarray(profile[1], np.float64)
        bs = np.ascontiguousarray(np.concatenate([np.asarray(profile[0], np.int32), np.zeros(1, np.int32)]), np.int32)
        check(_native.lib().dbi_shard_splitters_cost(_p(s), nshards, factor, bc.shape[0], _p(bs), _p(bc), _p(out)))
    return out[: nshards - 1]


def java_key(mass: np.ndarray, factor: int) -> np.ndarray:
    """(int)(mass * factor), Java semantics (truncation toward zero)."""
    return np.trunc(np.asarray(mass, np.float64) * float(factor)).astype(np.int64)


def owner_of(mass: np.ndarray, split: np.ndarray, factor: int) -> np.ndarray:
    """Owner shard of each mass: the number of splitter keys <= its key."""
    return np.searchsorted(np.asarray(split, np.int64), java_key(mass, factor), side="right")


def host_samples(masses: np.ndarray) -> np.ndarray:
    """Host twin of dbi_shard_samples over a dense record array (CPU tests):
    SHARD_SAMPLES evenly spaced masses + records per sample."""
    n = masses.shape[0]
    out = np.full(SHARD_SAMPLES + 1, np.nan)
    if n:
        idx = (np.arange(SHARD_SAMPLES, dtype=np.uint64) * np.uint64(n)) // np.uint64(SHARD_SAMPLES)
        out[:SHARD_SAMPLES] = masses[idx.astype(np.int64)]
        out[SHARD_SAMPLES] = n / SHARD_SAMPLES
    else:
        out[SHARD_SAMPLES] = 0.0
    return out


def concat_exports(parts: Sequence[dict]) -> dict:
    """The whole index from the owners' exports (Engine.export), in shard order."""
    if not parts:
        raise ValueError("no shards")
    out = {k: np.concatenate([p[k] for p in parts]) for k in ("mass", "prot_id", "offset", "length", "occ_prot")}
    occ, base = [np.zeros(1, np.uint64)], 0
    for p in parts:
        occ.append(p["occ_off"][1:].astype(np.uint64) + np.uint64(base))
        base += int(p["occ_off"][-1])
    out["occ_off"] = np.concatenate(occ)
    return out


def shard_stats(eng: Engine) -> DbiShardStats:
    st = DbiShardStats()
    check(_native.lib().dbi_shard_stats_get(eng.h, ctypes.byref(st)))
    return st


class ShardComm:
    """RCCL communicator of one rank (one process per GPU)."""

    def __init__(self, unique_id: bytes, nranks: int, rank: int, device: int):
        if len(unique_id) != 128:
            raise ValueError("RCCL unique id must be 128 bytes")
        self.nranks, self.rank, self.device = nranks, rank, device
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        h = ctypes.c_void_p()
        check(_native.lib().dbi_comm_init(buf, nranks, rank, device, ctypes.byref(h)))
        self.h = h

    @classmethod
    def host(cls, name: str, nranks: int, rank: int, device: int, slot_bytes: int = 64 << 20) -> "ShardComm":
        """TESTS ONLY: the host-staged transport (dbi_comm_init_host): the same
        collectives through POSIX shared memory ``name`` between the processes of
        one node, so N processes on ONE GPU run the N-rank driver."""
        self = cls.__new__(cls)
        self.nranks, self.rank, self.device = nranks, rank, device
        h = ctypes.c_void_p()
        check(_native.lib().dbi_comm_init_host(name.encode(), nranks, rank, device, slot_bytes, ctypes.byref(h)))
        self.h = h
        return self

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        check(_native.lib().dbi_comm_unique_id(buf))
        return bytes(buf)

    def allgatherv(self, d_send: int, d_recv: int, rank_bytes: Sequence[int]) -> None:
        rb = np.ascontiguousarray(rank_bytes, np.uint64)
        assert rb.shape[0] == self.nranks
        check(_native.lib().dbi_comm_allgatherv(self.h, ctypes.c_void_p(d_send) if d_send else None,
                                                ctypes.c_void_p(d_recv), _p(rb), None))

    def allreduce_u64(self, d_in: int, d_out: int, n: int) -> None:
        """Sum of n u64 over every rank, device to device (ncclAllReduce)."""
        check(_native.lib().dbi_comm_allreduce_u64(self.h, ctypes.c_void_p(d_in), ctypes.c_void_p(d_out), n, None))

    def close(self) -> None:
        if getattr(self, "h", None):
            _native.lib().dbi_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def build_sharded(eng: Engine, comm: ShardComm, d_res: int, n_res: int, d_off: int, n_prot: int,
                  p_begin: int, p_end: int) -> DbiShardStats:
    """All phases over RCCL (dbi_build_sharded): this rank's owner slice."""
    check(_native.lib().dbi_build_sharded(eng.h, comm.h, ctypes.c_void_p(d_res), n_res, ctypes.c_void_p(d_off),
                                          n_prot, p_begin, p_end))
    return shard_stats(eng)


def build_sharded_local(engines: Sequence[Engine], d_res: int, n_res: int, d_off: int, n_prot: int,
                        ranges: Sequence[Tuple[int, int]], profile=None, balance: bool = False,
                        split: Optional[np.ndarray] = None) -> np.ndarray:
    """Every shard's handle in this process (exchange by device copies): the
    phases of dbi_build_sharded one by one.  ``profile`` = (band_split,
    band_cost): cost-balanced splitters; ``balance``: the splitters follow the
    merge-cost profile engines[0] keeps and this build updates, as
    dbi_build_sharded does; ``split``: these owner splitters (a warm
    dbi_build_sharded reusing its split).  Returns the owner splitters."""
    n = len(engines)
    assert 1 <= n <= MAX_SHARDS and len(ranges) == n
    L = _native.lib()
    samples = np.zeros((n, SHARD_SAMPLES + 1), np.float64)
    for r, (eng, (b, e)) in enumerate(zip(engines, ranges)):
        check(L.dbi_shard_digest(eng.h, ctypes.c_void_p(d_res), n_res, ctypes.c_void_p(d_off), n_prot, b, e, r, n))
        row = np.zeros(SHARD_SAMPLES + 1, np.float64)
        check(L.dbi_shard_samples(eng.h, _p(row)))
        samples[r] = row
    # the split is held for a build of the same shape only: the
    # same residues, proteins and shard ranges as the build that held it
    shape = (int(n_res), int(n_prot), tuple((int(b), int(e)) for b, e in ranges))
    held = getattr(engines[0], "_split_held", None) if balance else None
    if split is not None:
        split = np.ascontiguousarray(split, np.int32)[: n - 1]
    elif held is not None and held[0] == shape and held[1].shape[0] == n - 1:
        split = held[1]  # the last two builds ran this split, balanced: keep it (dbi_build_sharded's hysteresis)
    elif balance:
        s = np.ascontiguousarray(samples, np.float64).reshape(n * (SHARD_SAMPLES + 1))
        out = np.zeros(max(n - 1, 1), np.int32)
        check(L.dbi_shard_splitters_profiled(engines[0].h, _p(s), n, _p(out)))
        split = out[: n - 1]
    else:
        split = splitters(samples, n, engines[0].cparams.mass_group_factor, profile)
    sp = np.ascontiguousarray(np.concatenate([split, np.zeros(1, np.int32)]), np.int32)
    for eng in engines:
        cnt = np.zeros(n, np.uint64)
        check(L.dbi_shard_partition(eng.h, _p(sp), _p(cnt)))
    hs = (ctypes.c_void_p * n)(*[e.h.value for e in engines])
    check(L.dbi_shard_exchange_local(hs, n))
    for eng in engines:
        check(L.dbi_shard_merge(eng.h))
    if balance:
        sts = [shard_stats(e) for e in engines]
        mms = np.array([st.merge_gpu_ms for st in sts], np.float64)
        recs = np.array([st.n_received for st in sts], np.uint64)
        sp = np.ascontiguousarray(np.concatenate([split, np.zeros(1, np.int32)]), np.int32)
        check(L.dbi_shard_cost_update(engines[0].h, n, _p(sp), _p(mms), _p(recs)))
        balanced = n > 1 and mms.min() > 0 and mms.max() <= SPLIT_HOLD * mms.mean()
        # as dbi_build_sharded: held when this build ran the previous build's
        # split (same shape) and its owners were balanced
        prev = getattr(engines[0], "_split_prev", None)
        same = prev is not None and prev[0] == shape and np.array_equal(prev[1], split)
        engines[0]._split_held = (shape, split.copy()) if balanced and same else None
        engines[0]._split_prev = (shape, split.copy())
    return split


def query_sharded(eng: Engine, comm: ShardComm, d_mass: int, d_tol: int, nq: int, d_first: int,
                  d_count: int) -> None:
    """This rank's batch against the sharded index (dbi_query_sharded): windows
    routed to their key owners over RCCL; ids of the whole index come back."""
    check(_native.lib().dbi_query_sharded(eng.h, comm.h, ctypes.c_void_p(d_mass), ctypes.c_void_p(d_tol), nq,
                                          ctypes.c_void_p(d_first), ctypes.c_void_p(d_count)))


def query_sharded_local(engines: Sequence[Engine], batches: Sequence[Tuple[np.ndarray, np.ndarray]]):
    """Every shard's batch routed between the handles of this process
    (dbi_query_sharded_local).  Returns [(first, count)] per shard, ids of the
    whole index."""
    from ._native import DeviceBuffer
    n = len(engines)
    assert len(batches) == n
    dev = engines[0].device
    bufs = []
    for m, t in batches:
        m = np.ascontiguousarray(m, np.float64)
        t = np.ascontiguousarray(np.broadcast_to(t, m.shape), np.float64)
        k = m.shape[0]
        bufs.append((DeviceBuffer.from_numpy(m, dev) if k else DeviceBuffer(8, dev),
                     DeviceBuffer.from_numpy(t, dev) if k else DeviceBuffer(8, dev),
                     DeviceBuffer(8 * max(k, 1), dev), DeviceBuffer(8 * max(k, 1), dev), k))
    arr = lambda i: (ctypes.c_void_p * n)(*[b[i].ptr for b in bufs])  # noqa: E731
    nq = np.array([b[4] for b in bufs], np.uint64)
    hs = (ctypes.c_void_p * n)(*[e.h.value for e in engines])
    check(_native.lib().dbi_query_sharded_local(hs, n, arr(0), arr(1), _p(nq), arr(2), arr(3)))
    return [(b[2].download(np.uint64, b[4]), b[3].download(np.uint64, b[4])) for b in bufs]


def replicate(eng: Engine, comm: ShardComm) -> None:
    """Every owner's slice onto every rank over RCCL (dbi_shard_replicate): the
    engine then holds the index of the whole proteome and queries locally."""
    check(_native.lib().dbi_shard_replicate(eng.h, comm.h))


def replicate_local(engines: Sequence[Engine]) -> None:
    """dbi_shard_replicate_local: the same between the handles of this process."""
    n = len(engines)
    hs = (ctypes.c_void_p * n)(*[e.h.value for e in engines])
    check(_native.lib().dbi_shard_replicate_local(hs, n))
