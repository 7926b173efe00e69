"""GPU: a FASTA *file* through the whole drop-in path — the library's parser
(dbi_fasta_read, DBIndexer.run's FastaReader, DBIndexer.java:546-616), the
device build and queries — against the oracle over the same proteome parsed
by the reference-semantics reader (fasta.iter_fasta), plus the reference's
rejection of a FASTA without any UniProt accession (DBIndexer.java:560-565)."""
from __future__ import annotations

import numpy as np
import pytest

from dbindex_amd import fasta
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref
from tests.helpers import assert_index_equal, assert_queries_equal, query_masses

pytestmark = pytest.mark.gpu


def _write_swissprot_style(path, pp, width_of=lambda i: 60 if i % 3 else 80):
    """SwissProt-style file: wrapped sequence lines of varying width, sp| / tr|
    headers and a few headers with no accession, CRLF on some lines, a blank
    line between some records."""
    with open(path, "w", newline="") as fh:
        for i in range(pp.n_proteins):
            if i % 17 == 5:
                head = f"PLAIN{i} protein without an accession"
            elif i % 5 == 0:
                head = f"tr|T{i:07d}|TRN{i}_HUMAN Unreviewed {i} OS=Homo sapiens OX=9606 GN=T{i} PE=4 SV=1"
            else:
                head = fasta.uniprot_header(i)
            eol = "\r\n" if i % 7 == 3 else "\n"
            fh.write(">" + head + eol)
            s = pp.sequence(i)
            w = width_of(i)
            for k in range(0, len(s), w):
                fh.write(s[k:k + w] + eol)
            if i % 11 == 4:
                fh.write(eol)


def _iter_parse(path):
    with open(path, newline="") as fh:
        items = list(fasta.iter_fasta(fh))
    seqs = [s for _, s in items]
    res, off = fasta.PackedProteins.from_sequences(seqs).residues, fasta.PackedProteins.from_sequences(seqs).offsets
    return items, res, off


@pytest.fixture(scope="module")
def engine_cls():
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    return Engine


@pytest.mark.parametrize("n", [1000, 20000])
def test_fasta_file_build_matches_oracle(engine_cls, tmp_path, n):
    pp = fasta.config("human").slice(0, n) if n > 1000 else fasta.config("1k")
    path = str(tmp_path / "db.fasta")
    _write_swissprot_style(path, pp)
    items, res, off = _iter_parse(path)
    assert len(items) == pp.n_proteins and "".join(s for _, s in items) == pp.residues.tobytes().decode()
    got = fasta.read_fasta(path)
    assert got.n_proteins == pp.n_proteins and np.array_equal(got.residues, res)
    assert np.array_equal(got.offsets, off)
    assert got.defs == [d.rstrip("\r") for d, _ in items]
    assert got.n_uniprot == sum(1 for d, _ in items if fasta.uniprot_accession(d))
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, res, off)
    with engine_cls(cp) as eng:
        eng.build(got)
        assert_index_equal(eng, oix, f"fasta file {n}")
        m, t = query_masses(oix, 5000, seed=11)
        assert_queries_equal(eng, oix, m, t, f"fasta file {n} queries")


@pytest.mark.parametrize("ptm", [False, True])
def test_fasta_file_registered_upload(engine_cls, tmp_path, ptm):
    """A parsed proteome above the upload's 16-MiB ring threshold: dbi_build
    pins the parser's own 2-MiB-page buffer and DMAs it directly (no staging
    copy), taking the parser's '[' finding for the inline-PTM decision; the
    same residues from a plain numpy copy go through the pinned ring.  Both
    indexes equal the oracle's."""
    pp = fasta.config("swissprot").slice(0, 60000)
    seqs = pp.sequences()
    if ptm:  # a few inline formulas far into the file (DBIndexer.java:288-303)
        for i in (41000, 52345, 59999):
            s = seqs[i]
            seqs[i] = s[:5] + "[HPO3]" + s[5:]
        pp = fasta.PackedProteins.from_sequences(seqs)
    path = str(tmp_path / "big.fasta")
    with open(path, "w") as fh:
        fasta.write_fasta(pp, fh)
    got = fasta.read_fasta(path, threads=8, with_defs=False)
    assert got.n_residues > (16 << 20) and np.array_equal(got.residues, pp.residues)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    copy = fasta.PackedProteins(np.array(got.residues), np.array(got.offsets))
    with engine_cls(cp) as eng:
        for src, what in ((got, "parser buffer"), (copy, "numpy copy"), (got, "parser buffer again")):
            eng.build(src)
            assert_index_equal(eng, oix, f"{what} ptm={ptm}")


@pytest.mark.parametrize("n,threads,ptm", [(1000, 0, False), (60000, 3, False), (60000, 16, False),
                                           (60000, 0, True)])
def test_build_fasta_one_call(engine_cls, tmp_path, n, threads, ptm):
    """dbi_build_fasta (the one-off build in one call: the parser's pinned
    residue buffer DMA'd straight to HBM) builds the oracle's index of the
    file, cold and warm, with the file's offsets and definitions handed back;
    a file with inline '[formula]' PTMs takes dbi_build's PTM path."""
    pp = fasta.config("1k") if n <= 1000 else fasta.config("swissprot").slice(0, n)
    if ptm:
        seqs = pp.sequences()
        for i in (7, n // 2, n - 1):
            seqs[i] = seqs[i][:5] + "[HPO3]" + seqs[i][5:]
        pp = fasta.PackedProteins.from_sequences(seqs)
    path = str(tmp_path / "fused.fasta")
    _write_swissprot_style(path, pp)
    items, res, off = _iter_parse(path)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, res, off)
    with engine_cls(cp) as eng:
        for phase in ("cold", "warm"):
            st, offs, defs = eng.build_fasta(path, threads=threads, with_defs=True)
            assert np.array_equal(offs, off) and defs == [d.rstrip("\r") for d, _ in items]
            assert st.n_total == oix.n_total
            assert_index_equal(eng, oix, f"build_fasta {n} t{threads} ptm={ptm} [{phase}]")
        m, t = query_masses(oix, 2000, seed=5)
        assert_queries_equal(eng, oix, m, t, f"build_fasta {n} queries")


def test_indexer_run_on_a_fasta_file(tmp_path):
    """DBIndexer.run(path): proteins in file order, ids = FASTA positions, the
    store answers like the oracle built from the reference-semantics parse."""
    from dbindex_amd.indexer import DBIndexer
    pp = fasta.config("1k").slice(0, 400)
    path = str(tmp_path / "db.fasta")
    _write_swissprot_style(path, pp)
    items, res, off = _iter_parse(path)
    prm = DBIndexSearchParams.trypsin(2)
    oix = cref.Index(prm.to_c(), res, off)
    ix = DBIndexer(prm)
    ix.init()
    ix.run(path)
    st = ix.indexStore
    assert st.getTotalSeqCount() == oix.n_total and st.getNumberSequences() == oix.n_keys
    u = oix.unique()
    seqs = [s for _, s in items]
    m, t = query_masses(oix, 60, seed=4)
    for mi, ti in zip(m, t):
        got = st.getSequences(float(mi), float(ti))
        want = oix.query(float(mi), float(ti))
        assert len(got) == len(want)
        for g, i in zip(got, want):
            p0, o, ln = int(u["prot_id"][i]), int(u["offset"][i]), int(u["length"][i])
            assert g.getSequence() == seqs[p0][o:o + ln] and g.getProteinIds()[0] == p0
            assert list(g.getProteinIds()) == [int(x) for x in u["occ_prot"][u["occ_off"][i]:u["occ_off"][i + 1]]]


def test_indexer_rejects_a_fasta_without_accessions(tmp_path):
    from dbindex_amd.indexer import DBIndexer, DBIndexerException
    path = str(tmp_path / "plain.fasta")
    with open(path, "w") as fh:
        for i, s in enumerate(fasta.config("1k").slice(0, 20).sequences()):
            fh.write(f">protein_{i} no accession here\n{s}\n")
    ix = DBIndexer(DBIndexSearchParams.trypsin(2))
    ix.init()
    with pytest.raises(DBIndexerException, match="Uniprot"):
        ix.run(path)
