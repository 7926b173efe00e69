"""Inline '[formula]' PTMs (DBIndexer.java:288-303), oracle side (CPU) and
engine vs oracle (GPU).

The reference walks the protein string and, at the first start whose walk
reaches a '[', adds the formula's mass as one more step (pepSize + 1; the
residue before it counted again by isEnzyme / checkCleavage), then removes
every copy of that bracketed formula from its local protein string, so every
later start sees the protein without it; offsets are in that stripped string
while peptide identity and text come from the ProteinCache's unstripped
string.  The oracle restates that loop literally (oracle/cpu_ref.cpp
cut_seq_literal); the engine strips the formulas on the host and walks the
formula-carrying proteins on the device (k_ptm_digest).  FormulaCalculator
(external jar) is restated as a monoisotopic element sum: parity unpinned.
"""
from __future__ import annotations

import numpy as np
import pytest

from dbindex_amd import fasta
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref

H2O_PROTON = DBIndexSearchParams().h2o_proton
MONO = DBIndexSearchParams().residue_mass
O_MASS = 15.99491461956


def _pack(seqs):
    lens = np.array([len(s) for s in seqs], np.uint64)
    off = np.zeros(len(seqs) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    return np.frombuffer("".join(seqs).encode(), np.uint8).copy(), off


def _digest(prm, seqs):
    res, off = _pack(seqs)
    d = cref.digest(prm.to_c(), res, off)
    return sorted(zip(d.pid.tolist(), d.offset.tolist(), d.length.tolist(), d.mass.tolist()))


def _mass(s):
    m = H2O_PROTON
    for c in s:
        m = m + MONO[c]
    return m


def test_oracle_formula_step_known_answer():
    """WWWWWK[O]WWWWWR, trypsin mc1: start 0 emits WWWWWK, then the formula step
    at the same end (K counted again: mc 1) emits WWWWWK + O at offset 0 length
    6; the formula is gone for start 6 (WWWWWR)."""
    got = _digest(DBIndexSearchParams.trypsin(1), ["WWWWWK[O]WWWWWR"])
    m6 = _mass("WWWWWK")
    want = sorted([(0, 0, 6, m6), (0, 0, 6, m6 + O_MASS), (0, 6, 6, _mass("WWWWWR"))])
    assert [(a, b, c) for a, b, c, _ in got] == [(a, b, c) for a, b, c, _ in want]
    assert np.allclose([x[3] for x in got], [x[3] for x in want], rtol=0, atol=1e-9)
    # mc 0: the double-counted K breaks the walk at the formula step
    got0 = _digest(DBIndexSearchParams.trypsin(0), ["WWWWWK[O]WWWWWR"])
    assert [(a, b, c) for a, b, c, _ in got0] == [(0, 0, 6), (0, 6, 6)]


def test_oracle_formula_reached_by_a_non_cleavage_start_is_dropped():
    """Far from the protein start the first walk to reach a formula starts at a
    non-cleavage position (no peptide): the result is the stripped protein's."""
    base = fasta.config("1k").sequence(3)
    k = 200
    with_ptm = base[:k] + "[HPO3]" + base[k:]
    prm = DBIndexSearchParams.trypsin(2)
    assert _digest(prm, [with_ptm]) == _digest(prm, [base])


def test_oracle_duplicate_formulas_vanish_with_the_first():
    """String.replace removes every copy of the bracketed formula at once."""
    prm = DBIndexSearchParams.trypsin(1)
    assert _digest(prm, ["WWWWWK[O]WWWWWR[O]GGGGGGK"]) == _digest(prm, ["WWWWWK[O]WWWWWRGGGGGGK"])


@pytest.mark.parametrize("seq", ["[O]PEPTIDEK", "PEPT[O"])
def test_oracle_reference_exceptions(seq):
    """A formula before the first residue (charAt(-1)) and '[' without ']'
    throw out of cutSeq in the reference: the oracle refuses the proteome."""
    with pytest.raises(ValueError):
        _digest(DBIndexSearchParams.trypsin(1), ["PEPTIDEKAAAAAAR", seq])


def test_oracle_unknown_element_ends_the_protein():
    """UnknownElementMassException is caught by cutSeq: the protein's later
    starts are skipped, earlier records stay, other proteins are untouched."""
    prm = DBIndexSearchParams.trypsin(1)
    a = "WWWWWKGGGGGGR" * 3
    got = _digest(prm, [a + "[Xq]" + a, a])
    p0 = [r for r in got if r[0] == 0]
    p1 = [r for r in got if r[0] == 1]
    assert p1 and len(p0) < len(p1) * 2 and p0 == [r for r in p0 if r[1] + r[2] <= len(a) + 1]


def ptm_proteome(n=150, seed=5):
    """A 1k slice with inline formulas: near protein starts (reached by
    cleavage starts), after K/R (double-counted), before P, adjacent pairs,
    repeated formulas, at the protein end, an unknown element."""
    rng = np.random.default_rng(seed)
    forms = ["O", "HPO3", "C2H2O", "CH2", "C2H3NO", "H-2O-1"]
    seqs = []
    for i, s in enumerate(fasta.config("1k").slice(0, n).sequences()):
        if i % 3 == 2:
            seqs.append(s)
            continue
        pts = sorted(set(rng.integers(1, len(s), size=int(rng.integers(1, 4))).tolist()))
        kr = [j + 1 for j, c in enumerate(s[:60]) if c in "KR" and j + 1 < len(s)]
        if kr and i % 2 == 0:
            pts = sorted(set(pts + kr[:2]))
        out, prev = [], 0
        for j, q in enumerate(pts):
            out.append(s[prev:q])
            f = forms[int(rng.integers(0, len(forms)))]
            out.append(f"[{f}]" + (f"[{forms[(j + 1) % len(forms)]}]" if i % 7 == 0 else ""))
            prev = q
        out.append(s[prev:])
        if i % 11 == 0:
            out.append("[O]")
        if i == 40:
            out.insert(2, "[Qx2]")
        seqs.append("".join(out))
    return seqs


@pytest.mark.gpu
@pytest.mark.parametrize("name,prm", [
    ("tryp2", DBIndexSearchParams.trypsin(2)),
    ("tryp1_nocutP", DBIndexSearchParams.trypsin(1, enzyme_nocut_residues="P")),
    ("semi1", DBIndexSearchParams.semi_tryptic(1)),
    ("mand", DBIndexSearchParams.trypsin(2, mandatory_internal_aas="C")),
])
def test_engine_ptm_matches_oracle(name, prm):
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    from tests.helpers import assert_index_equal, assert_queries_equal, query_masses
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    seqs = ptm_proteome()
    import re
    assert _digest(prm, seqs) != _digest(prm, [re.sub(r"\[[^\]]*\]", "", s) for s in seqs])  # the formulas matter
    res, off = _pack(seqs)
    cp = prm.to_c()
    oix = cref.Index(cp, res, off)
    pp = fasta.PackedProteins(res, off)
    with Engine(cp) as eng:
        for phase in ("cold", "warm"):
            eng.build(pp)
            assert_index_equal(eng, oix, f"ptm {name} [{phase}]")
        m, t = query_masses(oix, 5000, seed=3)
        assert_queries_equal(eng, oix, m, t, f"ptm {name} queries")


@pytest.mark.gpu
@pytest.mark.parametrize("seq", ["[O]PEPTIDEK", "PEPT[O"])
def test_engine_ptm_reference_exceptions(seq):
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    res, off = _pack(["PEPTIDEKAAAAAAR", seq])
    with Engine(DBIndexSearchParams.trypsin(1).to_c()) as eng:
        with pytest.raises(_native.DBIndexStoreException, match="StringIndexOutOfBounds"):
            eng.build(fasta.PackedProteins(res, off))


@pytest.mark.gpu
def test_store_ptm_text_from_the_cache_strings():
    """DBIndexer.run over proteins with formulas: the records come from the
    stripped walks, the text and flanks from the ProteinCache's strings (with
    their formulas) at those offsets, as IndexMerge.java:452-461 reads them."""
    from dbindex_amd import _native
    from dbindex_amd.indexer import DBIndexer
    from oracle import pyref
    from tests.helpers import query_masses
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    prm = DBIndexSearchParams.trypsin(2)
    seqs = ptm_proteome(60)
    items = [(fasta.uniprot_header(i), s) for i, s in enumerate(seqs)]
    res, off = _pack(seqs)
    oix = cref.Index(prm.to_c(), res, off)
    ix = DBIndexer(prm)
    ix.init()
    ix.run(items)
    st = ix.indexStore
    assert st.getTotalSeqCount() == oix.n_total and st.getNumberSequences() == oix.n_keys
    u = oix.unique()
    m, t = query_masses(oix, 80, seed=9)
    for mi, ti in zip(m, t):
        got = st.getSequences(float(mi), float(ti))
        ids = oix.query(float(mi), float(ti))
        assert len(got) == len(ids)
        for g, i in zip(got, ids):
            p0, o, ln = int(u["prot_id"][i]), int(u["offset"][i]), int(u["length"][i])
            assert g.getMass() == float(u["mass"][i]) and g.getProteinIds()[0] == p0
            assert g.getSequence() == seqs[p0][o:o + ln]
            assert (g.getResLeft(), g.getResRight()) == pyref.get_residues(o, ln, seqs[p0])


@pytest.mark.gpu
def test_engine_ptm_text_is_not_rebuilt_or_digested_on_device():
    """A build with inline formulas leaves the unstripped text resident:
    dbi_rebuild refuses it (it would digest the '[' characters as residues),
    and the device-input paths (dbi_build_device, dbi_count) refuse residues
    holding '[' instead of indexing them silently differently from dbi_build."""
    from dbindex_amd import _native
    from dbindex_amd._native import DeviceBuffer, synchronize
    from dbindex_amd.engine import Engine
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    seqs = ptm_proteome(40)
    res, off = _pack(seqs)
    pp = fasta.PackedProteins(res, off)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, res, off)
    from tests.helpers import assert_index_equal
    with Engine(cp) as eng:
        eng.build(pp)
        with pytest.raises(_native.DBIndexStoreException, match="dbi_rebuild after a build with inline"):
            eng.rebuild()
        eng.build(pp)  # the refusal left the handle usable
        assert_index_equal(eng, oix, "ptm build after refused rebuild")
        d_res = DeviceBuffer.from_numpy(np.concatenate([res, np.zeros(16, np.uint8)]), 0)
        d_off = DeviceBuffer.from_numpy(off.astype(np.uint64), 0)
        synchronize(0)
        for call in (lambda: eng.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins),
                     lambda: eng.count_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)):
            with pytest.raises(_native.DBIndexStoreException, match="device-resident residues"):
                call()
        # plain text on the same paths still builds
        plain = fasta.config("1k").slice(0, 50)
        eng.build(plain)
        st = eng.rebuild()
        assert st.n_total == cref.Index(cp, plain.residues, plain.offsets).n_total


def test_formula_mass_known_answers():
    """The independent Python restatement of FormulaCalculator against sums
    worked by hand (element masses written out), then the C++ oracle's
    (which the device walk mirrors) against it: bit-identical."""
    import math
    from oracle import pyref
    H, C, N, O, P = 1.00782503207, 12.0, 14.0030740048, 15.99491461956, 30.97376163
    kat = {
        "O": O,
        "H2O": 2 * H + O,
        "HPO3": ((H + P) + 3 * O),
        "C2H3NO": (((2 * C) + 3 * H) + N) + O,
        "H-2O-1": (-2 * H) + (-1 * O),
        "CH2": C + 2 * H,
        "C12": 12 * C,
    }
    for f, want in kat.items():
        assert pyref.formula_mass(f) == want, f
    for bad in ("Qx2", "2H", "O-", "h2o", "H2O]", "C2H3NO ", "Xx"):
        assert math.isnan(pyref.formula_mass(bad)), bad
    forms = list(kat) + ["Se", "NaCl", "C6H12O6", "C-2H-3", "Hg2Cl2", "SiO2", "H10", "D2O", "K1", "B4", "Zn0"]
    for f in forms + ["Qx2", "2H", "O-"]:
        a, b = pyref.formula_mass(f), cref.formula_mass(f)
        assert (math.isnan(a) and math.isnan(b)) or np.float64(a).view(np.uint64) == np.float64(b).view(np.uint64), f
