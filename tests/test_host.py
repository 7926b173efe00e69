"""CPU tests (no GPU): the C-ABI library loads and exports every symbol of
include/dbindex_hip.h, parameter packing, the DBIndexStore mirror's host-side
state machine and filters, the indexer's host checks, and the synthetic
FASTA generator / reader.  Nothing here launches a kernel.
"""
from __future__ import annotations

import ctypes
import io
import os
import re

import numpy as np
import pytest

from dbindex_amd import _native, fasta
from dbindex_amd.indexer import DBIndexer, DBIndexerException
from dbindex_amd.params import DBIndexSearchParams, DbiParams, MONO_RESIDUE_MASS
from dbindex_amd.store import DBIndexStoreHip, get_residues
from oracle import pyref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dbindex_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_ \*]*?\b(dbi_[a-z0-9_]+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    L = _native.lib()
    names = header_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    bound = {n for n, _, _ in _native.SIGNATURES}
    assert set(names) == bound, (set(names) ^ bound)


def test_abi_version_and_errors():
    L = _native.lib()
    assert L.dbi_abi_version() >= 1
    s = ctypes.c_void_p()
    bad = DBIndexSearchParams(index_factor=0).to_c()
    assert L.dbi_store_create(ctypes.byref(bad), 0, ctypes.byref(s)) == _native.DBI_E_INVALID
    assert b"index_factor" in L.dbi_last_error()


@pytest.mark.parametrize("mc,semi", [(0, 0), (2, 0), (2, 1)])
def test_params_default_matches_python(mc, semi):
    c = DbiParams()
    _native.lib().dbi_params_default(ctypes.byref(c), mc, semi)
    py = (DBIndexSearchParams.semi_tryptic(mc) if semi else DBIndexSearchParams.trypsin(mc)).to_c()
    assert bytes(c) == bytes(py)


def test_mass_table_literals():
    # monoisotopic residue masses pinned in DESIGN.md (AssignMass is absent from the reference)
    assert MONO_RESIDUE_MASS["G"] == 57.021464
    assert MONO_RESIDUE_MASS["W"] == 186.079313
    assert MONO_RESIDUE_MASS["K"] == 128.094963
    assert len([k for k in MONO_RESIDUE_MASS if k in fasta.CANONICAL]) == 20
    assert MONO_RESIDUE_MASS["I"] == MONO_RESIDUE_MASS["L"]


# ------------------------------------------------------------- store (host)
def test_store_state_machine_messages():
    st = DBIndexStoreHip(DBIndexSearchParams.trypsin(2))
    with pytest.raises(_native.DBIndexStoreException, match="not initialized"):
        st.startAddSeq()
    with pytest.raises(_native.DBIndexStoreException, match="Index path is missing"):
        st.init("")
    st.init("x.fasta_dbindex")
    with pytest.raises(_native.DBIndexStoreException, match="Already intialized"):
        st.init("x.fasta_dbindex")
    with pytest.raises(_native.DBIndexStoreException, match="Not in transaction"):
        st.stopAddSeq()
    st.startAddSeq()
    with pytest.raises(_native.DBIndexStoreException, match="In transaction already"):
        st.startAddSeq()
    assert not st.indexExists() and st.getNumberSequences() == 0 and st.getEntryKeys() == []
    st.close()


def test_store_filter_sequence_matches_reference_rule():
    for prm in [DBIndexSearchParams.trypsin(2), DBIndexSearchParams.trypsin(2, mandatory_internal_aas="CK")]:
        st = DBIndexStoreHip(prm)
        for m, seq in [(499.99, "AAAAAK"), (500.0, "AAAAAK"), (6000.0, "ACAAAK"), (6000.01, "ACAAAK"),
                       (800.0, "AAAAAC"), (800.0, "KAAAAA"), (800.0, "AAAAAA")]:
            assert st.filterSequence(m, seq) == pyref.filter_sequence(prm, m, seq), (m, seq)
        st.close()
    st = DBIndexStoreHip(DBIndexSearchParams.trypsin(2), device_digest=True)
    assert st.filterSequence(800.0, "AAAAAK") == _native.FILTER_SKIP_PROTEIN_START
    st.close()


def test_store_add_sequence_validation_and_drop_count():
    prm = DBIndexSearchParams.trypsin(2, index_factor=8)
    st = DBIndexStoreHip(prm)
    st.init("db")
    st.startAddSeq()
    assert st.addProteinDef(0, "sp|P1|A\tB", "PEPTIDEKAAAAAAK") == 0
    assert st.getProteinDef(0) == "sp|P1|A B"  # ProteinCache.addProtein tab -> space
    assert st.getProteinSequence(0) == "PEPTIDEKAAAAAAK" and st.getNumberProteins() == 1
    with pytest.raises(_native.DBIndexStoreException, match="protein numbers"):
        st.addProteinDef(5, "x", "AAA")
    st.addSequence(927.45, 0, 8, proteinId=0)
    st.addSequence(8000.5, 0, 8, proteinId=0)  # bucket 8 > NUM_BUCKETS-1: dropped, still counted
    assert st.getTotalSeqCount() == 2
    with pytest.raises(_native.DBIndexStoreException, match="outside its protein"):
        st.addSequence(927.45, 10, 8, proteinId=0)
    with pytest.raises(_native.DBIndexStoreException, match="addProteinDef"):
        st.addSequence(927.45, 0, 8, proteinId=3)
    st.close()


def test_get_residues_twins():
    prot = "MKWVTFISLLLLFSSAYSRGVFRR"
    for off in range(0, len(prot) - 6):
        for ln in (6, 7, 9):
            if off + ln > len(prot):
                continue
            r = get_residues(off, ln, prot)
            assert (r.getResLeft(), r.getResRight()) == pyref.get_residues(off, ln, prot)


# ------------------------------------------------------------- indexer (host)
def test_indexer_host_checks():
    prm = DBIndexSearchParams.trypsin(2)
    ix = DBIndexer(prm)
    with pytest.raises(RuntimeError, match="Not initialized"):
        ix.run([("sp|P1|X", "PEPTIDEK")])
    ix.init()
    with pytest.raises(RuntimeError, match="Already inited"):
        ix.init()
    with pytest.raises(DBIndexerException, match="Uniprot"):
        ix.run([("no accession here", "PEPTIDEK")])


# ------------------------------------------------------------- FASTA
def test_synthetic_deterministic_and_canonical():
    a = fasta.config("1k")
    b = fasta.config("1k")
    assert a.sha256() == b.sha256() and a.n_proteins == 1000
    lens = np.diff(a.offsets)
    assert lens.min() >= 30 and lens.max() <= 35000
    assert set(np.unique(a.residues).tobytes().decode()) <= set(fasta.CANONICAL)
    assert all(fasta.uniprot_accession(d) for d in a.defs[:50])
    assert fasta.config("human").n_proteins == 20000


def test_fasta_write_read_roundtrip(tmp_path):
    pp = fasta.config("1k").slice(0, 40)
    path = tmp_path / "syn.fasta"
    with open(path, "w") as fh:
        fasta.write_fasta(pp, fh)
    text = path.read_text()
    assert all(len(l) <= 60 for l in text.splitlines() if not l.startswith(">"))
    back = fasta.read_fasta(str(path))
    assert back.sha256() == pp.sha256() and back.defs == pp.defs


def test_slice_and_from_sequences():
    pp = fasta.config("1k")
    s = pp.slice(10, 20)
    assert s.sequences() == pp.sequences()[10:20]
    t = fasta.PackedProteins.from_sequences(s.sequences())
    assert np.array_equal(t.residues, s.residues) and np.array_equal(t.offsets, s.offsets)


def test_synth_proteome_twin_is_range_consistent():
    """The counter-based proteome (numpy twin of dbi_synth_proteome): any
    protein range is the matching slice of the whole, so ranks can generate
    their own ranges with no data movement."""
    t = fasta.synth_tables()
    assert t[0].shape == (4096,) and t[1].shape == (65536,)
    assert set(np.unique(t[1]).tobytes().decode()) == set(fasta.CANONICAL)
    whole = fasta.synth_proteome(11, 0, 700, 0, t)
    for a, n in ((0, 1), (123, 300), (699, 1)):
        base = fasta.synth_residue_base(11, a, t[0])
        assert base == int(whole.offsets[a])
        part = fasta.synth_proteome(11, a, n, base, t)
        assert np.array_equal(part.residues, whole.residues[int(whole.offsets[a]):int(whole.offsets[a + n])])
        assert np.array_equal(part.offsets, whole.offsets[a:a + n + 1] - whole.offsets[a])


FASTA_EDGE_CASES = [
    "",
    "no header at all\nACDE\n",
    ">only\n",
    ">a\nACD\nEFG\n>b\n\n>c\nKKK",                     # empty sequence, no final newline
    "junk before\n>x y z\r\nAC DE\r\n\tFG\r\n>y\r\n",      # CRLF, inner whitespace, text before the first record
    ">p1\nAAA>BBB\n>p2 desc > with >\nCC\n",              # '>' inside a line is a residue / part of the definition
    ">\nMK\n>>double\nRR\n",                               # empty definition, definition starting with '>'
]


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_native_fasta_parser_matches_iter_fasta(threads):
    texts = list(FASTA_EDGE_CASES)
    buf = io.StringIO()
    fasta.write_fasta(fasta.config("1k"), buf, width=37)
    texts.append(buf.getvalue())
    for t in texts:
        want = list(fasta.iter_fasta(io.StringIO(t)))
        got = fasta.parse_fasta(t, threads=threads)
        assert got.n_proteins == len(want), (t[:40], got.n_proteins, len(want))
        assert got.defs == [d for d, _ in want]
        assert got.sequences() == [s for _, s in want]
        assert got.n_uniprot == sum(fasta.uniprot_accession(d) is not None for d, _ in want)


def test_native_fasta_parser_random_layouts(tmp_path):
    """Seeded random FASTA texts against iter_fasta: records whose lines and
    whitespace (spaces, tabs, CR, VT, FF, blank lines) fall at every offset of
    the parser's 64-byte blocks, '>' inside sequence lines and definitions,
    empty records, with and without a final newline; parsed from memory and
    read from a file (mapped), on 1 and 5 threads."""
    rng = np.random.default_rng(17)
    ws = [" ", "\t", "\r", "\x0b", "\x0c", "\n", "\n\n", "\r\n"]
    for case in range(12):
        parts = [] if case % 3 else ["preamble line\n"]
        for r in range(int(rng.integers(1, 60))):
            d = "".join(rng.choice(list("ABC|x >"), int(rng.integers(0, 30))))
            parts.append(">" + d + ("\r\n" if rng.random() < 0.2 else "\n"))
            n = int(rng.integers(0, 400))
            seq = []
            for _ in range(n):
                seq.append(str(rng.choice(list("ACDEFGHIKLMNPQRSTVWY>"), p=[0.0495] * 20 + [0.01])))
                if rng.random() < 0.04:
                    seq.append(str(rng.choice(ws)))
                if rng.random() < 1 / 61:
                    seq.append("\n")
            parts.append("".join(seq) + ("\n" if rng.random() < 0.8 else ""))
        t = "".join(parts)
        if rng.random() < 0.5:
            t = t.rstrip("\n")
        want = list(fasta.iter_fasta(io.StringIO(t)))
        path = tmp_path / f"r{case}.fasta"
        path.write_bytes(t.encode())
        for threads in (1, 5):
            for got in (fasta.parse_fasta(t, threads=threads), fasta.read_fasta(str(path), threads=threads)):
                assert got.n_proteins == len(want), (case, threads)
                assert got.defs == [d for d, _ in want]
                assert got.sequences() == [s for _, s in want], (case, threads)


def test_native_fasta_read_file(tmp_path):
    pp = fasta.config("1k")
    path = tmp_path / "p.fasta"
    with open(path, "w") as fh:
        fasta.write_fasta(pp, fh)
    back = fasta.read_fasta(str(path), threads=4)
    assert np.array_equal(back.residues, pp.residues) and np.array_equal(back.offsets, pp.offsets)
    assert back.defs == pp.defs and back.n_uniprot == pp.n_proteins
    with pytest.raises(_native.DBIndexStoreException):
        fasta.read_fasta(str(tmp_path / "missing.fasta"))


def test_index_file_matches_header(tmp_path):
    """dbi_index_file_matches (host only): missing / foreign files never match."""
    p = DBIndexSearchParams.trypsin(2).to_c()
    v = ctypes.c_int(7)
    _native.check(_native.lib().dbi_index_file_matches(ctypes.byref(p), str(tmp_path / "none").encode(), ctypes.byref(v)))
    assert v.value == 0
    junk = tmp_path / "junk.dbihip"
    junk.write_bytes(b"NOTANIDX" + bytes(200))
    _native.check(_native.lib().dbi_index_file_matches(ctypes.byref(p), str(junk).encode(), ctypes.byref(v)))
    assert v.value == 0


def test_static_mods_semantics():
    """SearchParamReader.java:401-583 via AssignMassToStaticParam (:7-14):
    f <= 0 ignored, otherwise added to the residue mass; N15 scales f, except
    cysteine (f + e*(f - 57.02146f)); terminus parameters set cTerm/nTerm."""
    base = DBIndexSearchParams.trypsin(2)
    q = base.with_static_mods({"C": 57.02146, "M": 0.0, "K": -1.0}, cterm=1.5, nterm=2.5)
    assert q.residue_mass["C"] == base.residue_mass["C"] + 57.02146
    assert q.residue_mass["M"] == base.residue_mass["M"] and q.residue_mass["K"] == base.residue_mass["K"]
    assert (q.cterm, q.nterm) == (1.5, 2.5) and (base.cterm, base.nterm) == (0.0, 0.0)
    n = base.with_static_mods({"C": 57.02146, "S": 79.966331}, n15_enrichment=0.5)
    assert n.residue_mass["S"] == base.residue_mass["S"] + 79.966331 * 0.5
    assert n.residue_mass["C"] == base.residue_mass["C"] + (57.02146 + 0.5 * (57.02146 - float(np.float32(57.02146))))
    # no C mod under N15: f = 0 + e*(0 - 57.02146f) < 0 -> ignored
    assert base.with_static_mods({}, n15_enrichment=0.5).residue_mass["C"] == base.residue_mass["C"]
    with pytest.raises(ValueError):
        base.with_static_mods({"J": 1.0})


def test_protein_cache_and_decoy_accession():
    """ProteinCache (ProteinCache.java:60-127) and the string the decoy regexp
    is matched against (DBIndexer.java:608-611)."""
    from dbindex_amd.store import ProteinCache
    pc = ProteinCache()
    assert not pc.isPopulated()
    assert pc.addProtein("sp|P1|A\tB", "PEPTIDEK") == 0
    assert pc.addProtein("sp|P2|C", "MKR") == 1
    assert pc.getProteinDef(0) == "sp|P1|A B" and pc.getNumberProteins() == 2
    assert pc.getPeptideSequence(0, 2, 4) == "PTID"
    assert pc.getPeptideSequence(1, 1, 5) is None  # substring out of range: logged, null
    assert pc.getProteinSequence(5) is None
    assert fasta.fasta_accession("sp|P12345|NAME_HUMAN desc") == "P12345"
    assert fasta.fasta_accession("Reverse_sp|P12345|NAME_HUMAN desc") == "Reverse_sp|P12345|NAME_HUMAN"
    assert fasta.fasta_accession("") == ""
