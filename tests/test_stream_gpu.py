"""GPU parity of the count-only streaming path (BASELINE.json configs[4]):
the device proteome generator equals its numpy twin byte for byte, and the
COUNT-mode digest equals the oracle's cutSeq occurrence count (totalSeqCount)
on the same proteins, and the full build's n_total."""
from __future__ import annotations

import numpy as np
import pytest

from dbindex_amd import fasta
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine():
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    return Engine


TABLES = fasta.synth_tables()


def _download(d_res, n_res, d_off, n_prot):
    from dbindex_amd._native import check, lib
    import ctypes
    res = np.zeros(n_res, np.uint8)
    off = np.zeros(n_prot + 1, np.uint64)
    check(lib().dbi_dev_copy_d2h(0, res.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(d_res), n_res))
    check(lib().dbi_dev_copy_d2h(0, off.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(d_off), 8 * (n_prot + 1)))
    return res, off


@pytest.mark.parametrize("seed,p0,n", [(4, 0, 1000), (4, 123457, 3001), (9, 7, 1)])
def test_synth_matches_numpy_twin(Engine, seed, p0, n):
    base = fasta.synth_residue_base(seed, p0, TABLES[0])
    ref = fasta.synth_proteome(seed, p0, n, base, TABLES)
    with Engine(DBIndexSearchParams.trypsin(2)) as eng:
        d_res, d_off, n_res = eng.synth_proteome(seed, p0, n, base, TABLES)
        assert n_res == ref.n_residues
        res, off = _download(d_res, n_res, d_off, n)
    assert np.array_equal(off, ref.offsets)
    assert np.array_equal(res, ref.residues)


@pytest.mark.parametrize("name,prm,n", [
    ("nonspec", DBIndexSearchParams.non_specific(50), 120),
    ("tryp2", DBIndexSearchParams.trypsin(2), 2000),
    ("semi2", DBIndexSearchParams.semi_tryptic(2), 400),
    ("tryp2_drop", DBIndexSearchParams.trypsin(2, index_factor=8, max_precursor_mass=9000.0), 2000),
])
def test_count_matches_oracle(Engine, name, prm, n):
    base = fasta.synth_residue_base(4, 5000, TABLES[0])
    pp = fasta.synth_proteome(4, 5000, n, base, TABLES)
    cp = prm.to_c()
    dg = cref.digest(cp, pp.residues, pp.offsets)
    want_total, want_drop = dg.mass.shape[0], int(dg.dropped.sum())
    with Engine(cp) as eng:
        d_res, d_off, n_res = eng.synth_proteome(4, 5000, n, base, TABLES)
        for _ in range(2):
            total, dropped = eng.count_device(d_res, n_res, d_off, n)
            assert (total, dropped) == (want_total, want_drop), name
        st = eng.build(pp)
        assert st.n_total == want_total and st.n_dropped == want_drop
        # a count after a build on the same engine (workspace reuse)
        d_res, d_off, n_res = eng.synth_proteome(4, 5000, n, base, TABLES)
        assert eng.count_device(d_res, n_res, d_off, n) == (want_total, want_drop)


def test_count_empty(Engine):
    with Engine(DBIndexSearchParams.non_specific(50)) as eng:
        d_res, d_off, n_res = eng.synth_proteome(4, 0, 0, 0, TABLES)
        assert n_res == 0
        assert eng.count_device(d_res, 0, d_off, 0) == (0, 0)


@pytest.mark.parametrize("shift", [1, 3, 8, 13])
def test_count_and_build_misaligned_residues(shift):
    """The C-ABI takes any device pointer: residues starting at an odd byte
    (chunks packed back to back) must count and index exactly as aligned ones."""
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    pp = fasta.config("1k").slice(0, 120)
    for prm in (DBIndexSearchParams.non_specific(50), DBIndexSearchParams.trypsin(2)):
        cp = prm.to_c()
        oix = cref.Index(cp, pp.residues, pp.offsets)
        buf = np.full(pp.n_residues + shift + 64, ord("W"), np.uint8)  # heavy bytes around the data
        buf[shift:shift + pp.n_residues] = pp.residues
        d_res = _native.DeviceBuffer.from_numpy(buf, 0)
        d_off = _native.DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), 0)
        with Engine(cp, 0) as eng:
            tot, drop = eng.count_device(d_res.ptr + shift, pp.n_residues, d_off.ptr, pp.n_proteins)
            assert (tot, drop) == (oix.n_total, oix.n_dropped), (shift, prm)
            st = eng.build_device(d_res.ptr + shift, pp.n_residues, d_off.ptr, pp.n_proteins)
            assert st.n_total == oix.n_total and st.n_unique == oix.n_unique, (shift, prm)
