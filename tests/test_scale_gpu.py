"""GPU parity at BASELINE.json scale (configs[2]-[4]).

* configs[2]: the full SwissProt-scale proteome (560k proteins, seed 3,
  trypsin mc2) built on the device and compared with the oracle bit-exactly
  (every count, every mass bit, the unique table, the occurrence CSR, the
  entry keys) plus 1M +-20 ppm queries.
* configs[3]: semi-tryptic mc2 on a 30k-protein slice of the same proteome
  (the 1024-thread big-chunk tier reached) + 1M queries vs the oracle; the FULL
  semi-tryptic build (~1e9 occurrences) through size-independent properties:
  masses sorted, occurrence offsets monotone and ending at n_kept, protein
  ids in range, n_total equal to the COUNT-mode digest.
* configs[4]: non-specific 6-50 COUNT parity (totalSeqCount) on samples of
  the 50M-protein counter-based proteome at p0 = 0, 25M, 49.99M and across
  the global 2^32-residue seam, generated on the device.

The oracle runs multi-threaded here (cref.threads: same results, it is the
checker); reference: DBIndexer.java:237-405, DBIndexStoreSQLiteByteIndexMerge
.java:620-719, DBIndexStoreSQLiteMult.java:315-350.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from dbindex_amd import fasta
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref
from dbindex_amd._native import DeviceBuffer
from tests.helpers import assert_index_equal, assert_queries_equal, query_masses

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share is 16


@pytest.fixture(scope="module")
def Engine():
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    return Engine


@pytest.fixture(scope="module")
def swissprot():
    return fasta.config("swissprot", with_defs=False)


@pytest.fixture(scope="module")
def swissprot_oix(swissprot):
    """The oracle's index of configs[2] (built once for the tests below)."""
    cp = DBIndexSearchParams.trypsin(2).to_c()
    with cref.threads(THREADS):
        return cref.Index(cp, swissprot.residues, swissprot.offsets)


def test_swissprot_full_tryptic(Engine, swissprot, swissprot_oix):
    """configs[2] at full size: 560k proteins, 201M residues, 54M peptides."""
    pp = swissprot
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = swissprot_oix
    with cref.threads(THREADS):
        m, t = query_masses(oix, 1_000_000)
        with Engine(cp) as eng:
            st = eng.build(pp)
            assert st.n_total > 50_000_000
            assert_index_equal(eng, oix, "swissprot tryptic mc2")
            assert_queries_equal(eng, oix, m, t, "swissprot 1M queries")
            # a second (warm, bounded-digest) build of the same input
            eng.build(pp)
            assert_index_equal(eng, oix, "swissprot tryptic mc2 [warm]")


def test_swissprot_sharded_8_shards(Engine, swissprot, swissprot_oix):
    """configs[2] in its sharded form: the whole proteome split by residues
    into 8 protein ranges (8 handles on this GPU, dbi_shard_exchange_local:
    the phases of an 8-rank dbi_build_sharded), every record routed to the
    owner of its mass key and merged there (IndexMerge.getMergedData,
    DBIndexStoreSQLiteByteIndexMerge.java:620-719, across shards); the owners'
    slices concatenated equal the oracle's single index array for array, then
    the replicated index (north star's all-gatherv) on every handle equals it
    too and answers 200k queries."""
    from dbindex_amd import _native, shard
    pp = swissprot
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = swissprot_oix
    o = oix.unique()
    k = 8
    d_res = _native.DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), 0)
    d_off = _native.DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), 0)
    engines = [Engine(cp, 0) for _ in range(k)]
    try:
        for rep in ("cold", "warm"):
            shard.build_sharded_local(engines, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins,
                                      shard.protein_ranges(pp.offsets, k))
            sts = [shard.shard_stats(e) for e in engines]
            assert sum(s.n_total for s in sts) == oix.n_total
            assert sum(s.n_received for s in sts) == oix.n_kept
            assert sum(s.n_unique for s in sts) == oix.n_unique and sum(s.n_keys for s in sts) == oix.n_keys
            assert min(s.n_received for s in sts) > oix.n_kept // (2 * k)  # owners balanced by the splitters
            g = shard.concat_exports([e.export() for e in engines])
            assert np.array_equal(g["mass"].view(np.uint64), o["mass"].view(np.uint64)), rep
            for key in ("prot_id", "offset", "length", "occ_off", "occ_prot"):
                assert np.array_equal(g[key].astype(np.uint64), o[key].astype(np.uint64)), (rep, key)
            del g
        shard.replicate_local(engines)
        with cref.threads(THREADS):
            m, t = query_masses(oix, 200_000, seed=13)
            for r in (0, k - 1):
                assert_index_equal(engines[r], oix, f"swissprot replica {r}/{k}")
                assert_queries_equal(engines[r], oix, m, t, f"swissprot replica {r}/{k} queries")
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("big_split,semi_part", [("auto", 1), ("1", 1), ("auto", 0)])
def test_swissprot_semi_slice(Engine, swissprot, big_split, semi_part):
    """configs[3] parity on a 30k-protein slice (~55M semi-tryptic peptides),
    large enough to reach the 1024-thread big-chunk tier (equal-mass spikes).
    option big_split=1: the big tier in its two size classes (512-thread blocks
    for chunks of up to 3968 records, the rest 1024-thread), which the engine
    otherwise uses only for lists longer than 1024 chunks (full semi-tryptic).
    Warm builds partition their records by the first LSD digit in the digest
    (semi_part=1: part_hist / bin_scatter, then the radix tail's third pass),
    or run the radix tail's three passes (semi_part=0); a timed warm build
    shows which stages ran."""
    pp = swissprot.slice(0, 30000)
    cp = DBIndexSearchParams.semi_tryptic(2).to_c()
    opts = {"semi_part": semi_part}
    if big_split != "auto":
        opts["big_split"] = int(big_split)
    with cref.threads(THREADS):
        oix = cref.Index(cp, pp.residues, pp.offsets)
        m, t = query_masses(oix, 1_000_000)
        with Engine(cp, options=opts) as eng:
            for phase in ("cold", "warm", "replay", "timed"):
                eng.set_timing(phase == "timed")
                st = eng.build(pp)
                assert st.n_big_bins > 0, "slice too small to reach the big-chunk tier"
                assert_index_equal(eng, oix, f"semi slice [{phase}, big split {big_split}, semi_part {semi_part}]")
            names = {name for name, _, _ in eng.stage_times()}
            if semi_part:
                assert {"part_hist", "bin_scatter", "radix_scatter"} <= names, names
            else:
                assert "bin_scatter" not in names and "radix_scatter" in names, names
            assert_queries_equal(eng, oix, m, t, "semi slice 1M queries")


def _download(ptr: int, dtype, n: int) -> np.ndarray:
    from dbindex_amd._native import check, lib
    out = np.zeros(n, dtype)
    if n:
        check(lib().dbi_dev_copy_d2h(0, out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), out.nbytes))
    return out


def test_swissprot_semi_full_properties(Engine, swissprot):
    """configs[3] at full size (~1e9 occurrences, ~110 GB of HBM at peak):
    too big for the oracle, so size-independent properties of the index."""
    from dbindex_amd._native import DeviceBuffer, synchronize
    pp = swissprot
    cp = DBIndexSearchParams.semi_tryptic(2).to_c()
    d_res = DeviceBuffer.from_numpy(pp.residues)
    d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64))
    synchronize()
    with Engine(cp) as eng:
        total, dropped = eng.count_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)
        st = eng.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)
        assert st.n_total == total and st.n_dropped == dropped and st.n_total > 900_000_000
        assert st.n_kept == st.n_total - st.n_dropped and 0 < st.n_unique <= st.n_kept
        v = eng.device_view()
        U, K = st.n_unique, st.n_kept
        step = 1 << 26
        prev_m, prev_o = -np.inf, 0
        nkeys = 0
        prev_key = None
        for a in range(0, U, step):
            n = min(step, U - a)
            mass = _download(v.mass + 8 * a, np.float64, n)
            occ = _download(v.occ_off + 4 * a, np.uint32, n)
            ln = _download(v.length + 4 * a, np.uint32, n)
            pid = _download(v.prot_id + 4 * a, np.uint32, n)
            assert mass[0] >= prev_m and np.all(np.diff(mass) >= 0), "masses not sorted"
            assert np.all(np.isfinite(mass)) and mass.min() >= 500.0 and mass.max() <= 6000.0
            assert occ[0] >= prev_o and np.all(np.diff(occ.astype(np.int64)) >= 1), "occurrence offsets"
            assert np.all(ln >= 6) and np.all(pid < pp.n_proteins)
            keys = (mass * 10000.0).astype(np.int64)
            nkeys += int(np.count_nonzero(np.diff(keys))) + (1 if prev_key is None or keys[0] != prev_key else 0)
            prev_m, prev_o, prev_key = mass[-1], int(occ[-1]), keys[-1]
        assert _download(v.occ_off + 4 * U, np.uint32, 1)[0] == K
        assert nkeys == st.n_keys  # one row per distinct mass key (buckets: 1000-Da edges are key edges)
        # occurrence protein ids in range (strided sample of the CSR)
        occ_pid = _download(v.occ_prot, np.uint32, min(K, 1 << 24))
        assert occ_pid.max() < pp.n_proteins


TREMBL_P = 50_000_000
TABLES = fasta.synth_tables()


def _seam_protein(seed: int) -> int:
    """First protein whose residues cross global residue index 2^32."""
    lt = TABLES[0]
    lo = (1 << 32) // 400
    base = fasta.synth_residue_base(seed, lo, lt)
    lens = fasta.synth_lengths(seed, lo, 1 << 22, lt)
    cum = base + np.cumsum(lens.astype(np.int64))
    assert base <= (1 << 32) < int(cum[-1])
    return lo + int(np.searchsorted(cum, 1 << 32, side="right"))  # starts <= 2^32, ends past it


@pytest.mark.parametrize("where", ["start", "middle", "end", "seam_2^32"])
def test_trembl_count_samples(Engine, where):
    """configs[4]: non-specific 6-50 totalSeqCount of 2500 proteins of the
    50M-protein synthetic proteome, generated on the device at the sample's
    place, equals the oracle's cutSeq count of the numpy twin."""
    seed, n = 4, 2500
    p0 = {"start": 0, "middle": 25_000_000, "end": TREMBL_P - n, "seam_2^32": None}[where]
    if p0 is None:
        p0 = _seam_protein(seed) - n // 2
    base = fasta.synth_residue_base(seed, p0, TABLES[0])
    pp = fasta.synth_proteome(seed, p0, n, base, TABLES)
    if where == "seam_2^32":
        assert base < (1 << 32) < base + pp.n_residues
    cp = DBIndexSearchParams.non_specific(50).to_c()
    with cref.threads(THREADS):
        want = cref.count(cp, pp.residues, pp.offsets)
    with Engine(cp) as eng:
        d_res, d_off, n_res = eng.synth_proteome(seed, p0, n, base, TABLES)
        assert n_res == pp.n_residues
        assert eng.count_device(d_res, n_res, d_off, n) == want
        # per SQLiteMult bucket (DBIndexStoreSQLiteMult.java:215-217), accumulated over two calls
        with cref.threads(THREADS):
            hist = cref.count_buckets(cp, pp.residues, pp.offsets)
        d_hist = DeviceBuffer.from_numpy(np.zeros(cp.index_factor + 1, np.uint64))
        assert eng.count_buckets_device(d_res, n_res, d_off, n, d_hist.ptr) == want
        assert eng.count_buckets_device(d_res, n_res, d_off, n, d_hist.ptr) == want
        assert np.array_equal(d_hist.download(np.uint64, cp.index_factor + 1), 2 * hist)
