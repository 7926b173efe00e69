"""GPU parity of SEARCH_UNINDEXED (DBIndexer.cutAndSearch, DBIndexer.java:707-747,
over MassRangeFilteringIndex, MassRangeFilteringIndex.java:40-130) against the
oracle's restatement (oracle/cref.cut_and_search, pinned to the walk-level
pyref.cut_and_search in tests/test_oracle.py): the same set of sequences, and
per sequence the first occurrence's mass bits, offset, length, cutSeq flanks
and the protein ids without repeats.  The reference returns THashMap order;
ours is ascending mass, so the comparison is by sequence.
"""
from __future__ import annotations

import numpy as np
import pytest

from dbindex_amd import _native, fasta
from dbindex_amd.indexer import DBIndexer, IndexerMode
from dbindex_amd.params import DBIndexSearchParams, tolerance_in_dalton
from dbindex_amd.store import MassRange, MassRangeFilteringIndexHip
from oracle import cref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")


def _as_dict(lst):
    out = {}
    for s in lst:
        assert s.getSequence() not in out, "a sequence twice in one result"
        out[s.getSequence()] = (s.getMass(), s.getSequenceOffset(), s.getSequenceLen(), s.getResLeft(),
                                s.getResRight(), list(s.getProteinIds()))
    return out


def _same(res, exp, ctx):
    got = _as_dict(res)
    assert got.keys() == exp.keys(), (ctx, len(got), len(exp))
    for k, e in exp.items():
        g = got[k]
        assert np.float64(g[0]).view(np.uint64) == np.float64(e[0]).view(np.uint64), (ctx, k)
        assert g[1:] == e[1:], (ctx, k, g, e)
    masses = [s.getMass() for s in res]
    assert masses == sorted(masses), ctx


def _ranges(pp, prm, rng, k):
    d = cref.digest(prm.to_c(), pp.residues, pp.offsets)
    pick = d.mass[rng.integers(0, d.mass.shape[0], k)]
    tol = rng.choice([0.0, 0.004, 0.05, 1.0, 40.0], k)
    return pick, tol


RESIDENT, STREAM = MassRangeFilteringIndexHip.RESIDENT, MassRangeFilteringIndexHip.STREAM


def _indexer(prm, pp, mode=RESIDENT):
    ix = DBIndexer(prm, IndexerMode.SEARCH_UNINDEXED, indexStore=MassRangeFilteringIndexHip(prm, mode=mode))
    ix.init()
    ix.run(pp)
    return ix


@pytest.mark.parametrize("mode", [RESIDENT, STREAM], ids=["resident", "stream"])
@pytest.mark.parametrize("name,prm,nprot", [
    ("tryp2", DBIndexSearchParams.trypsin(2), 1000),
    ("semi2", DBIndexSearchParams.semi_tryptic(2), 200),
    ("nonspec", DBIndexSearchParams.non_specific(30), 40),
    ("mandK", DBIndexSearchParams.trypsin(2, mandatory_internal_aas="K"), 1000),
    ("no_drop", DBIndexSearchParams.trypsin(4, max_precursor_mass=9500.0), 500),
])
def test_cut_and_search_parity(name, prm, nprot, mode):
    pp = fasta.config("1k").slice(0, nprot)
    ix = _indexer(prm, pp, mode)
    rng = np.random.default_rng(11)
    cp = prm.to_c()
    for k in (1, 4, 25):
        m, t = _ranges(pp, prm, rng, k)
        exp = cref.cut_and_search(cp, pp.residues, pp.offsets, m, t)
        res = ix.getSequences([MassRange(a, b) for a, b in zip(m.tolist(), t.tolist())])
        _same(res, exp, (name, k))
        assert ix.indexStore.getNumberSequences() == len(exp)
    # single-range entry points
    m0 = float(m[0])
    _same(ix.getSequencesUsingDaltonTolerance(m0, 0.5), cref.cut_and_search(cp, pp.residues, pp.offsets,
                                                                            [m0], [0.5]), (name, "Da"))
    tppm = tolerance_in_dalton(m0, 10.0)
    _same(ix.getSequencesUsingPPMTolerance(m0, 10.0), cref.cut_and_search(cp, pp.residues, pp.offsets,
                                                                          [m0], [tppm]), (name, "ppm"))
    if name == "no_drop":  # peptides past NUM_BUCKETS*BUCKET_MASS_RANGE are searchable here
        exp = cref.cut_and_search(cp, pp.residues, pp.offsets, [8700.0], [800.0])
        assert any(v[0] >= 8000.0 for v in exp.values())
        _same(ix.getSequences([MassRange(8700.0, 800.0)]), exp, (name, "past 8000"))


@pytest.mark.parametrize("mode", [RESIDENT, STREAM], ids=["resident", "stream"])
def test_cut_and_search_edges(mode):
    prm = DBIndexSearchParams.trypsin(2)
    pp = fasta.config("1k").slice(0, 300)
    ix = _indexer(prm, pp, mode)
    cp = prm.to_c()
    st = ix.indexStore
    assert not st.indexExists()
    with pytest.raises(_native.DBIndexStoreException):
        st.getEntryKeys()
    # no ranges, NaN, negative, past every peptide, one huge window
    for m, t in ([], []), ([float("nan")], [1.0]), ([-3.0], [1.0]), ([7.0e4], [5.0]), ([3000.0], [3000.0]):
        exp = cref.cut_and_search(cp, pp.residues, pp.offsets, m, t)
        _same(ix.getSequences([MassRange(a, b) for a, b in zip(m, t)]), exp, ("edge", m, t))
        assert st.getNumberSequences() == len(exp)
    # residues come from the sequence itself
    res = ix.getSequencesUsingDaltonTolerance(1500.0, 5.0)
    assert res
    s = res[0]
    prot = ix.getProteins(s)[0]
    r = st.getResidues(s, prot)
    assert (r.getResLeft(), r.getResRight()) == (s.getResLeft(), s.getResRight())


@pytest.mark.parametrize("mode", [RESIDENT, STREAM], ids=["resident", "stream"])
def test_unindexed_duplicates_within_and_across_proteins(mode):
    prm = DBIndexSearchParams.trypsin(0, min_precursor_mass=300.0)
    seqs = ["MPEPTIDEKAAGGKPEPTIDEK", "GGGKPEPTIDEK", "PEPTIDEKW"] * 3
    pp = fasta.PackedProteins.from_sequences(seqs)
    ix = _indexer(prm, pp, mode)
    from dbindex_amd.params import calculate_mass
    mass = calculate_mass("PEPTIDEK", prm)
    res = ix.getSequencesUsingDaltonTolerance(mass, 0.0)
    exp = cref.cut_and_search(prm.to_c(), pp.residues, pp.offsets, [mass], [0.0])
    _same(res, exp, "dups")
    assert _as_dict(res)["PEPTIDEK"][5] == list(range(9))


def test_unindexed_store_rules():
    prm = DBIndexSearchParams.trypsin(2)
    st = MassRangeFilteringIndexHip(prm)
    with pytest.raises(_native.DBIndexStoreException):
        st.setDeviceDigest(False)
    import ctypes
    from dbindex_amd.store import DBIndexStoreHip
    other = DBIndexStoreHip(prm)
    other.init("x")
    out = ctypes.POINTER(_native.DbiSeqList)()
    with pytest.raises(_native.DBIndexStoreException, match="SEARCH_UNINDEXED"):
        _native.check(_native.lib().dbi_store_cut_and_search(other.s, None, None, 0, ctypes.byref(out)))
    other.close()
    st.close()


@pytest.mark.parametrize("name,prm,nprot", [
    ("tryp2", DBIndexSearchParams.trypsin(2), 1000),         # fused / count-emit digest (bounded is off)
    ("semi2", DBIndexSearchParams.semi_tryptic(2), 300),
    ("nonspec50", DBIndexSearchParams.non_specific(50), 300),
])
def test_window_filtered_build_is_the_full_index_restricted(name, prm, nprot):
    """dbi_set_windows: the filtered build's unique table, occurrence lists
    and order equal the unbucketed full build's rows whose mass lies in a
    window -- and dbi_rebuild over the resident inputs gives the same."""
    from dbindex_amd.engine import Engine
    pp = fasta.config("1k").slice(0, nprot)
    rng = np.random.default_rng(5)
    with Engine(prm.to_c(), 0) as full, Engine(prm.to_c(), 0) as filt:
        full.set_bucket_drop(False)
        filt.set_bucket_drop(False)
        full.build(pp)
        g = full.export()
        um = g["mass"]
        for rep, k in enumerate((1, 7, 60)):
            m = um[rng.integers(0, um.shape[0], k)] + rng.normal(0, 0.01, k)
            t = rng.choice([0.0, 0.02, 0.5, 3.0], k)
            filt.set_windows(m, t)
            st = filt.build(pp) if rep == 0 else filt.rebuild()
            f = filt.export()
            sel = np.zeros(um.shape[0], bool)
            for a, b in zip(m - t, m + t):
                sel |= (um >= a) & (um <= b)
            ids = np.nonzero(sel)[0]
            assert st.n_unique == ids.shape[0], (name, k)
            assert np.array_equal(f["mass"].view(np.uint64), um[ids].view(np.uint64)), (name, k)
            for key in ("prot_id", "offset", "length"):
                assert np.array_equal(f[key], g[key][ids]), (name, k, key)
            occ = [g["occ_prot"][g["occ_off"][i]:g["occ_off"][i + 1]] for i in ids]
            exp_occ = np.concatenate(occ) if occ else np.zeros(0, g["occ_prot"].dtype)
            assert np.array_equal(f["occ_prot"], exp_occ), (name, k)
        # the filter off again: the full index
        filt.set_windows(on=False)
        filt.rebuild()
        assert np.array_equal(filt.export()["mass"].view(np.uint64), um.view(np.uint64))
