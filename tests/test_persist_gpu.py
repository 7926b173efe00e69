"""GPU: a built index on disk and back (dbi_index_save / dbi_index_load) and
the DBIndexStore mirror's indexExists reuse contract (DBIndexer.java:522-527):
the loaded index answers exactly like the oracle's."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from dbindex_amd import fasta
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref
from tests.helpers import assert_index_equal, assert_queries_equal, query_masses

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine():
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    return Engine


def test_engine_save_load_roundtrip(Engine, tmp_path):
    from dbindex_amd import _native
    pp = fasta.config("1k")
    prm = DBIndexSearchParams.trypsin(2)
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    path = str(tmp_path / "idx.dbihip")
    with Engine(cp) as a:
        a.build(pp)
        a.save(path)
    with Engine(cp) as b:
        st = b.load(path)
        assert st.n_total == oix.n_total and st.n_unique == oix.n_unique
        assert_index_equal(b, oix, "loaded")
        m, t = query_masses(oix, 1500)
        assert_queries_equal(b, oix, m, t, "loaded")
        # a loaded index saves again byte for byte
        b.save(str(tmp_path / "again.dbihip"))
    assert open(path, "rb").read() == open(tmp_path / "again.dbihip", "rb").read()
    # other parameters: the file is refused, loudly
    with Engine(DBIndexSearchParams.trypsin(1).to_c()) as c:
        with pytest.raises(_native.DBIndexStoreException):
            c.load(path)
    # a format-01 file (the FNV-1a tie order of round 2) is neither reused nor
    # loaded: its equal-mass ties would be ordered unlike a fresh build's
    old = bytearray(open(path, "rb").read())
    assert old[:8] == b"DBIHIP02"
    old[6:8] = b"01"
    p01 = str(tmp_path / "v01.dbihip")
    open(p01, "wb").write(bytes(old))
    def matches(pth):
        v = ctypes.c_int(-1)
        _native.check(_native.lib().dbi_index_file_matches(ctypes.byref(cp), pth.encode(), ctypes.byref(v)))
        return v.value
    assert matches(p01) == 0 and matches(path) == 1
    with Engine(cp) as d:
        with pytest.raises(_native.DBIndexStoreException):
            d.load(p01)


def test_store_persist_and_reuse(tmp_path):
    from dbindex_amd.indexer import DBIndexer
    from dbindex_amd.store import DBIndexStoreHip
    pp = fasta.config("1k").slice(0, 300)
    prm = DBIndexSearchParams.trypsin(2)
    name = str(tmp_path / "db.fasta")
    oix = cref.Index(prm.to_c(), pp.residues, pp.offsets)
    m, t = query_masses(oix, 300)

    def answers(ix):
        out = []
        for mm, tt in zip(m[:60], t[:60]):
            out.append(sorted((s.getSequence(), tuple(sorted(set(p.getId() for p in ix.getProteins(s)))))
                              for s in ix.getSequencesUsingDaltonTolerance(float(mm), float(tt))))
        return out

    # what the oracle answers: every unique peptide of the window, its proteins
    u = oix.unique()
    seqs = pp.sequences()
    want = []
    for mm, tt in zip(m[:60], t[:60]):
        rows = []
        for i in oix.query(float(mm), float(tt)):
            p0, o, ln = int(u["prot_id"][i]), int(u["offset"][i]), int(u["length"][i])
            prots = u["occ_prot"][u["occ_off"][i]:u["occ_off"][i + 1]]
            rows.append((seqs[p0][o:o + ln], tuple(sorted(set(int(x) for x in prots)))))
        want.append(sorted(rows))
    assert sum(len(w) for w in want) > 0

    first = DBIndexer(prm, indexStore=DBIndexStoreHip(prm, persist=True), database_name=name)
    first.init()
    assert not first.indexStore.indexExists()
    first.run(pp)
    assert answers(first) == want
    n_keys = first.getNumParentMasses()
    # a new process-like store with the same parameters finds the file and skips indexing
    second = DBIndexer(prm, indexStore=DBIndexStoreHip(prm, persist=True), database_name=name)
    second.init()
    assert second.indexStore.indexExists()
    second.run(iter(()))  # would raise "no UniProt accession" if it indexed
    assert answers(second) == want
    assert second.getNumParentMasses() == n_keys
    # other parameters: not reused
    other = DBIndexer(DBIndexSearchParams.trypsin(1),
                      indexStore=DBIndexStoreHip(DBIndexSearchParams.trypsin(1), persist=True), database_name=name)
    other.init()
    assert not other.indexStore.indexExists()


def test_unbucketed_or_filtered_index_is_not_saved(tmp_path):
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    pp = fasta.config("1k").slice(0, 50)
    with Engine(DBIndexSearchParams.trypsin(2).to_c(), 0) as eng:
        eng.set_bucket_drop(False)
        eng.build(pp)
        with pytest.raises(_native.DBIndexStoreException, match="bucketed"):
            eng.save(str(tmp_path / "x.dbihip"))
        eng.set_bucket_drop(True)
        eng.build(pp)
        eng.save(str(tmp_path / "x.dbihip"))
        eng.set_bucket_drop(False)
        with pytest.raises(_native.DBIndexStoreException, match="bucketed"):
            eng.load(str(tmp_path / "x.dbihip"))


@pytest.mark.parametrize("damage", ["truncate", "grow", "header_n_unique", "header_def_bytes", "occ_off",
                                    "mass_order", "prot_id", "occ_prot", "offset", "def_off"])
def test_damaged_index_file_is_refused(Engine, tmp_path, damage):
    """index_load checks the header against the file size before allocating and
    every content invariant of a build (occ_off monotone ending at n_kept,
    protein ids < P, peptide inside its protein, masses ascending, finite and in
    [1, 65536)): a damaged file is an error, never an out-of-range read."""
    import struct
    from dbindex_amd import _native
    pp = fasta.config("1k").slice(0, 100)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    path = str(tmp_path / "idx.dbihip")
    with Engine(cp) as a:
        st = a.build(pp)
        a.save(path)
    raw = bytearray(open(path, "rb").read())
    R, P, U, K = st.n_residues, st.n_proteins, st.n_unique, st.n_kept
    base = 128 + R + 16 * (P + 1)  # header, residues, offsets, def_off (no definitions)
    mass0, pid0, off0, len0 = base, base + 8 * U, base + 12 * U, base + 16 * U
    occ_off0, occ0 = base + 20 * U, base + 20 * U + 4 * (U + 1)
    if damage == "truncate":
        raw = raw[:-7]
    elif damage == "grow":
        raw += b"\0" * 8
    elif damage == "header_n_unique":
        struct.pack_into("<Q", raw, 8 + 8 + 8 + 16, 1 << 40)  # n_unique
    elif damage == "header_def_bytes":
        struct.pack_into("<Q", raw, 8 + 8 + 8 + 56, 1 << 50)  # def_bytes
    elif damage == "occ_off":
        struct.pack_into("<I", raw, occ_off0 + 4 * (U // 2), 0)
    elif damage == "mass_order":
        struct.pack_into("<d", raw, mass0 + 8 * (U // 2), 7000.0)
    elif damage == "prot_id":
        struct.pack_into("<I", raw, pid0 + 4 * 3, P + 5)
    elif damage == "occ_prot":
        struct.pack_into("<I", raw, occ0 + 4 * (K - 1), 0xFFFFFFF0)
    elif damage == "offset":
        struct.pack_into("<I", raw, off0 + 4 * 7, 1 << 20)
    elif damage == "def_off":  # definition offsets without definitions (def_bytes = 0)
        struct.pack_into("<Q", raw, 128 + R + 8 * (P + 1) + 8 * (P // 2), 1000)
    open(path, "wb").write(bytes(raw))
    with Engine(cp) as b:
        with pytest.raises(_native.DBIndexStoreException):
            b.load(path)
        b.build(pp)  # the engine stays usable
        assert b.stats().n_unique == U
