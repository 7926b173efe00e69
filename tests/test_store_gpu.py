"""GPU parity of the Java-API mirror (DBIndexer / DBIndexStore over the C-ABI
``dbi_store_*``) against the oracle: every field of every IndexedSequence a
query returns (sequence, mass bits, proteinIds in order, flanks, offset,
length), the store counters, entry keys / parent masses, ppm and multi-range
queries, getProteins(String), and the golden fixtures.

Reference flows: DBIndexer.run/cutSeq (DBIndexer.java:237-405,508-684),
DBIndexStoreSQLiteMult (:245-350), IndexMerge.getSequences/parseAddPeptideInfo
(:146-217,386-481), Util.getResidues (:130-162).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from dbindex_amd import fasta
from dbindex_amd.indexer import DBIndexer
from dbindex_amd.params import DBIndexSearchParams, calculate_mass, tolerance_in_dalton
from dbindex_amd.store import DBIndexStoreHip, MassRange
from oracle import cref, pyref
from tests.helpers import query_masses

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    from dbindex_amd import _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")


def expected(oix, seqs, ids):
    u = oix.unique()
    out = []
    for i in ids:
        pids = [int(x) for x in u["occ_prot"][u["occ_off"][i]:u["occ_off"][i + 1]]]
        p0, off, ln = int(u["prot_id"][i]), int(u["offset"][i]), int(u["length"][i])
        assert pids[0] == p0
        left, right = pyref.get_residues(off, ln, seqs[p0])
        out.append((seqs[p0][off:off + ln], float(u["mass"][i]), pids, left, right, off, ln))
    return out


def got(lst):
    return [(s.getSequence(), s.getMass(), list(s.getProteinIds()), s.getResLeft(), s.getResRight(),
             s.getSequenceOffset(), s.getSequenceLen()) for s in lst]


def same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x[0] == y[0] and np.float64(x[1]).view(np.uint64) == np.float64(y[1]).view(np.uint64)
        assert x[2:] == y[2:], (x, y)


def _indexer(prm, pp):
    ix = DBIndexer(prm)
    ix.init()
    ix.run(pp)
    return ix


@pytest.mark.parametrize("name,prm,nprot", [
    ("tryp2", DBIndexSearchParams.trypsin(2), 150),
    ("semi1", DBIndexSearchParams.semi_tryptic(1), 40),
    ("tryp1_if6", DBIndexSearchParams.trypsin(1, index_factor=6, enzyme_nocut_residues="P"), 150),
])
def test_indexer_device_digest(name, prm, nprot):
    pp = fasta.config("1k").slice(0, nprot)
    seqs = pp.sequences()
    oix = cref.Index(prm.to_c(), pp.residues, pp.offsets)
    ix = _indexer(prm, pp)
    st = ix.indexStore
    assert st.indexExists()
    assert st.getTotalSeqCount() == oix.n_total
    assert st.getNumberSequences() == oix.n_keys == ix.getNumParentMasses()
    keys = list(oix.entry_keys())
    assert st.getEntryKeys() == keys
    assert ix.getParentMasses() == [k * 1.0 / prm.mass_group_factor for k in keys]
    m, t = query_masses(oix, 150, seed=11)
    for mi, ti in zip(m, t):
        same(got(ix.getSequencesUsingDaltonTolerance(float(mi), float(ti))),
             expected(oix, seqs, oix.query(float(mi), float(ti))))


def test_store_host_digest_flow():
    """The reference's own flow: cutSeq -> filterSequence -> addSequence per
    peptide (the oracle's cutSeq drives the store), then stopAddSeq builds."""
    prm = DBIndexSearchParams.trypsin(2, index_factor=3000, max_precursor_mass=7999.0)
    pp = fasta.config("1k").slice(0, 120)
    seqs = pp.sequences()
    oix = cref.Index(prm.to_c(), pp.residues, pp.offsets)
    st = DBIndexStoreHip(prm)
    st.init("synthetic.fasta_dbindex")
    st.startAddSeq()
    for i, s in enumerate(seqs):
        assert st.addProteinDef(i, pp.defs[i], s) == i
    for (mass, pid, off, ln, _dropped) in pyref.digest(prm, seqs):
        assert st.filterSequence(mass, seqs[pid][off:off + ln]) == 0
        st.addSequence(mass, off, ln, proteinId=pid)
    st.stopAddSeq()
    assert oix.n_dropped > 0
    assert st.getTotalSeqCount() == oix.n_total
    assert st.getNumberSequences() == oix.n_keys and st.getEntryKeys() == list(oix.entry_keys())
    m, t = query_masses(oix, 100, seed=3)
    for mi, ti in zip(m, t):
        same(got(st.getSequences(float(mi), float(ti))), expected(oix, seqs, oix.query(float(mi), float(ti))))
    st.close()


def test_ppm_multirange_and_proteins():
    prm = DBIndexSearchParams.trypsin(2)
    pp = fasta.config("1k").slice(0, 200)
    seqs = pp.sequences()
    oix = cref.Index(prm.to_c(), pp.residues, pp.offsets)
    ix = _indexer(prm, pp)
    u = oix.unique()
    for i in range(0, oix.n_unique, max(1, oix.n_unique // 60)):
        mi = float(u["mass"][i])
        tol = tolerance_in_dalton(mi, 10.0)
        res = got(ix.getSequencesUsingPPMTolerance(mi, 10.0))
        base = expected(oix, seqs, oix.query(mi, tol))
        # the ppm path = the Dalton window plus the upper-bound probe loop (DBIndexer.java:787-844)
        assert [r[0] for r in res[:len(base)]] == [b[0] for b in base]
        assert len({r[0] for r in res}) == len(res)
        # single range delegates to getSequences(m, tol); >1 range reproduces the key-column binding
        same(got(ix.getSequences([MassRange(mi, 0.02)])), expected(oix, seqs, oix.query(mi, 0.02)))
        j = (i * 7 + 3) % oix.n_unique
        mj = float(u["mass"][j])
        same(got(ix.getSequences([MassRange(mi, 0.02), MassRange(mj, 0.5)])),
             expected(oix, seqs, oix.query_ranges([mi, mj], [0.02, 0.5])))
        # getProteins(String): exact-mass lookup + string equality (DBIndexer.java:925-947)
        pep = seqs[int(u["prot_id"][i])][int(u["offset"][i]):int(u["offset"][i]) + int(u["length"][i])]
        assert calculate_mass(pep, prm) == mi
        pids = {int(x) for x in u["occ_prot"][u["occ_off"][i]:u["occ_off"][i + 1]]}
        assert {p.getId() for p in ix.getProteins(pep)} == pids


@pytest.mark.parametrize("fname,prm,nprot", [
    ("golden_1k_tryp0.npz", DBIndexSearchParams.trypsin(0), 1000),
    ("golden_1k_tryp2.npz", DBIndexSearchParams.trypsin(2), 300),
])
def test_engine_matches_golden(fname, prm, nprot):
    from dbindex_amd.engine import Engine
    g = np.load(os.path.join(GOLDEN, fname))
    pp = fasta.config("1k") if nprot == 1000 else fasta.config("1k").slice(0, nprot)
    assert bytes(g["residues_sha256"]).decode() == pp.sha256()
    with Engine(prm.to_c()) as eng:
        eng.build(pp)
        st = eng.stats()
        assert st.n_total == int(g["n_total"][0]) and st.n_keys == int(g["n_keys"][0])
        ex = eng.export()
        assert np.array_equal(ex["mass"].view(np.uint64), g["u_mass"].view(np.uint64))
        for k, gk in [("prot_id", "u_pid"), ("offset", "u_offset"), ("length", "u_length"),
                      ("occ_off", "u_occ_off"), ("occ_prot", "u_occ_prot")]:
            assert np.array_equal(ex[k].astype(np.uint64), g[gk].astype(np.uint64)), k
        assert np.array_equal(eng.entry_keys().astype(np.int64), g["entry_keys"].astype(np.int64))
        first, count = eng.query(g["q_mass"], g["q_tol"])
        assert np.array_equal(first.astype(np.uint64), g["q_first"].astype(np.uint64))
        assert np.array_equal(count.astype(np.uint64), g["q_count"].astype(np.uint64))


def test_concurrent_store_queries_mixed_ranges():
    """Several host threads on one store: single-range getSequences(m, tol),
    multi-range getSequences(List<MassRange>) (the key-range path) and engine
    batch queries at once; every answer equals the oracle's (the query-side
    calls serialise on the handle's query lock and scratch)."""
    import threading
    prm = DBIndexSearchParams.trypsin(2)
    pp = fasta.config("1k").slice(0, 300)
    seqs = pp.sequences()
    oix = cref.Index(prm.to_c(), pp.residues, pp.offsets)
    ix = _indexer(prm, pp)
    st = ix.indexStore
    u = oix.unique()
    m, t = query_masses(oix, 400, seed=5)
    single = [expected(oix, seqs, oix.query(float(a), float(b))) for a, b in zip(m[:40], t[:40])]
    pairs = [(float(u["mass"][i]), float(u["mass"][(i * 7 + 3) % oix.n_unique]))
             for i in range(0, oix.n_unique, max(1, oix.n_unique // 40))]
    multi = [expected(oix, seqs, oix.query_ranges([a, b], [0.02, 0.5])) for a, b in pairs]
    of, oc = oix.query_batch(m, t)
    errors = []

    def run_single():
        for _ in range(5):
            for (a, b), want in zip(zip(m[:40], t[:40]), single):
                try:
                    same(got(st.getSequences(float(a), float(b))), want)
                except AssertionError:
                    errors.append("single")

    def run_multi():
        for _ in range(5):
            for (a, b), want in zip(pairs, multi):
                try:
                    same(got(st.getSequences([MassRange(a, 0.02), MassRange(b, 0.5)])), want)
                except AssertionError:
                    errors.append("multi")

    def run_batch():
        from dbindex_amd.engine import Engine
        eng = Engine.__new__(Engine)  # a view of the store's engine handle (not owned)
        eng.h, eng.device = st.engine_handle(), 0
        for _ in range(20):
            f, c = eng.query(m, t)
            if not (np.array_equal(c, oc) and np.array_equal(f[oc > 0], of[oc > 0])):
                errors.append("batch")
        eng.h = None

    th = [threading.Thread(target=f) for f in (run_single, run_multi, run_batch, run_single, run_multi)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]


def _with_decoys(pp, every):
    """FASTA items with a reversed-sequence ``Reverse_`` decoy after every
    ``every``-th target (every=0: all decoys at the end)."""
    seqs = pp.sequences()
    tg = [(pp.defs[i], s) for i, s in enumerate(seqs)]
    dec = [("Reverse_" + d, s[::-1]) for d, s in tg]
    if every == 0:
        return tg + dec
    out = []
    for i, x in enumerate(tg):
        out.append(x)
        if i % every == 0:
            out.append(dec[i])
    return out


def _pack(seqs):
    lens = np.array([len(s) for s in seqs], np.uint64)
    off = np.zeros(len(seqs) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    return np.frombuffer("".join(seqs).encode(), np.uint8).copy(), off


@pytest.mark.parametrize("every", [0, 3])
def test_decoy_regexp_protein_numbering(every):
    """DBIndexer.run with discardDecoyRegexp (DBIndexer.java:594-616): every
    protein enters the ProteinCache, only non-decoys are cut, so ids count the
    non-decoys while the store resolves text, flanks and definitions through
    the cache (IndexMerge.java:452-461, SQLiteMult.java:297/:457).  With
    decoys interleaved the answers come from shifted cache entries, exactly as
    the reference's; with decoys appended they are the target-only index."""
    prm = DBIndexSearchParams.trypsin(2, discard_decoy_regexp="^Reverse_")
    pp = fasta.config("1k").slice(0, 90)
    items = _with_decoys(pp, every)
    all_defs = [d for d, _ in items]
    all_seqs = [s for _, s in items]
    targets = [s for d, s in items if not d.startswith("Reverse_")]
    res, off = _pack(targets)
    oix = cref.Index(prm.to_c(), res, off)
    ix = DBIndexer(prm)
    ix.init()
    ix.run(items)
    assert ix.decoyDiscarded == len(items) - len(targets) > 0
    st = ix.indexStore
    assert st.getTotalSeqCount() == oix.n_total and st.getNumberSequences() == oix.n_keys
    u = oix.unique()
    m, t = query_masses(oix, 120, seed=17)
    n_shifted = n_raised = 0
    for mi, ti in zip(m, t):
        ids = oix.query(float(mi), float(ti))
        want, raises = [], False
        for i in ids:
            pids = [int(x) for x in u["occ_prot"][u["occ_off"][i]:u["occ_off"][i + 1]]]
            p0, o, ln = int(u["prot_id"][i]), int(u["offset"][i]), int(u["length"][i])
            cp = all_seqs[p0]
            if o > len(cp):
                raises = True
                break
            text = cp[o:o + ln] if o + ln <= len(cp) else None
            n_shifted += text != targets[p0][o:o + ln]
            left, right = pyref.get_residues(o, ln, cp)
            want.append((text, float(u["mass"][i]), pids, left, right, o, ln))
        if raises:
            n_raised += 1
            with pytest.raises(Exception, match="out of range"):
                st.getSequences(float(mi), float(ti))
            continue
        res_q = st.getSequences(float(mi), float(ti))
        same(got(res_q), want)
        for s in res_q[:3]:
            assert [p.getAccession() for p in st.getProteins(s)] == [all_defs[p] for p in s.getProteinIds()]
    if every == 0:
        assert n_shifted == 0 and n_raised == 0  # decoys after the targets: ids and cache agree
    else:
        assert n_shifted > 0  # the reference's shifted resolution is what is reproduced
