"""GPU: depth bins (warm lean builds).

A warm tryptic build partitions its records inside the digest by the high
digit of an equal-depth mass-bin map (sampled from the previous index), sorts
them into bins with one radix pass over the low digit, and bins every chunk
again in LDS.  The map is only a heuristic: whatever it is -- the previous
index of another proteome, a map that crowds one region past its capacity --
every build must equal the oracle (reference: DBIndexer.java:237-405,
DBIndexStoreSQLiteByteIndexMerge.java:620-719).
"""
from __future__ import annotations

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


def _stages(eng):
    return {name for name, _, _ in eng.stage_times()}


@pytest.mark.parametrize("depth,reuse", [(1, 1), (1, 0), (0, 1)])
def test_depth_warm_builds_match_oracle(Engine, depth, reuse):
    """Human scale (configs[1], 1.9M records): cold, then warm builds -- every
    stage timed (no graph), then untimed (captured, replayed) -- each equal to
    the oracle; with option depth_bins=0 the radix tail runs instead.  The map
    is sampled again only when the index changes size (option
    depth_map_reuse=0: every build)."""
    pp = fasta.config("human")
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    with Engine(cp, options={"depth_bins": depth, "depth_map_reuse": reuse}) as eng:
        eng.build(pp)
        assert "bin_scatter" not in _stages(eng)  # cold: the bounded digest's slot count, then the radix tail
        assert_index_equal(eng, oix, "cold")
        for k in range(3):
            eng.build(pp)
            names = _stages(eng)
            assert ("bin_scatter" in names) == (depth == 1), names
            assert ("radix_scatter" in names) == (depth == 0), names
            if depth and k == 2:  # (k = 0 is a redo, whose stage table starts after the map)
                assert ("depth_map" in names) == (reuse == 0), names
            assert_index_equal(eng, oix, f"warm timed {k}")
        eng.set_timing(False)
        for k in range(4):
            eng.build(pp)
            assert_index_equal(eng, oix, f"warm untimed {k}")
        m, t = query_masses(oix, 5000, seed=3)
        assert_queries_equal(eng, oix, m, t, "queries")


def test_depth_map_of_another_proteome(Engine):
    """The map comes from the resident index.  Proteome B (the same proteins
    rewritten over G/A/S/K/R: light peptides) built after A uses A's map: its
    records crowd the low high-digit regions past their capacity, the build
    is redone by the radix tail (ERR_PART) and the next takes depth bins over
    B's own map.  Then back to A.  Every build equals its oracle."""
    hum = fasta.config("human")
    a = hum.slice(0, 12000)
    light = np.frombuffer(b"GASKR", np.uint8)
    b_res = light[a.residues % 5].copy()
    b = fasta.PackedProteins(b_res, a.offsets.copy(), a.defs)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oa, ob = cref.Index(cp, a.residues, a.offsets), cref.Index(cp, b.residues, b.offsets)
    assert ob.n_total > 20000
    with Engine(cp) as eng:
        for k, (p, o) in enumerate([(a, oa), (a, oa), (b, ob), (b, ob), (b, ob), (a, oa), (a, oa)]):
            eng.build(p)
            assert_index_equal(eng, o, f"build {k}")
            if k in (1, 3, 4, 6):  # the map of the same proteome: depth bins
                assert "bin_scatter" in _stages(eng), (k, _stages(eng))
            if k in (2, 5):  # the other proteome's map overflows a region: redone by the radix tail
                assert "radix_scatter" in _stages(eng) and "bin_scatter" not in _stages(eng), (k, _stages(eng))
        m, t = query_masses(oa, 3000, seed=9)
        assert_queries_equal(eng, oa, m, t, "queries after the map changes")


@pytest.mark.parametrize("opts", [{}, {"big_split": 1}, {"big_side": 0}, {"big_side": 0, "big_split": 1}],
                         ids=["side", "side_split", "inline", "inline_split"])
def test_depth_equal_mass_spikes(Engine, opts):
    """Equal-mass spikes (a protein block rewritten as GAAAAAAK repeats) land
    whole in one depth bin: a chunk far above the LDS capacity, through the
    big / giant tiers from the bin-ordered records, warm and replayed -- the
    big tier beside the chunk sort (option big_side, default) or in line,
    in one size class or two (big_split)."""
    a = fasta.config("human").slice(0, 6000)
    spike = a.residues.copy()
    e = int(a.offsets[400])
    spike[:e] = np.resize(np.frombuffer(b"GAAAAAAK", np.uint8), e)
    c = fasta.PackedProteins(spike, a.offsets.copy(), a.defs)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oc = cref.Index(cp, c.residues, c.offsets)
    with Engine(cp, options=opts) as eng:
        eng.set_timing(False)
        for k in range(5):
            eng.build(c)
            assert_index_equal(eng, oc, f"spiked build {k} {opts}")


def test_options_and_cold_builds(Engine):
    """dbi_set_option refuses an unknown name or a value out of range
    (DBI_E_INVALID, the handle stays usable); dbi_set_cold makes the next build
    a cold one (the bounded digest's slot count, then its pass into exactly
    that, and the radix tail), after which warm builds
    take depth bins again -- every build equal to the oracle."""
    from dbindex_amd._native import DBIndexStoreException
    pp = fasta.config("human").slice(0, 8000)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    with Engine(cp) as eng:
        with pytest.raises(DBIndexStoreException, match="INVALID"):
            eng.set_option("no_such_option", 1)
        with pytest.raises(DBIndexStoreException, match="INVALID"):
            eng.set_option("chunk_target", 1 << 20)
        with pytest.raises(DBIndexStoreException, match="INVALID"):
            eng.set_option("test_fail", 3)  # a string option given a number
        for k in range(3):
            eng.build(pp)
            assert_index_equal(eng, oix, f"before cold {k}")
        assert "bin_scatter" in _stages(eng)
        eng.set_cold()
        eng.build(pp)
        names = _stages(eng)
        assert "digest_slots" in names and "digest" in names and "radix_scatter" in names, names
        assert "bin_scatter" not in names and "digest_emit" not in names, names
        assert_index_equal(eng, oix, "cold again")
        for k in range(3):
            eng.build(pp)
            assert_index_equal(eng, oix, f"after cold {k}")
        assert "bin_scatter" in _stages(eng)


def test_semi_first_digit_partition(Engine):
    """Warm semi-specific builds partition their records in the digest by the
    low digit of their linear fine bin (the radix tail's first LSD pass, fused:
    part_hist / bin_scatter, then the remaining radix pass).  Proteome A, then
    B: A with a block of GAAAAAAK repeats, whose equal-mass records crowd one
    region past the capacity A's counts gave it (ERR_PART: redone by the radix
    tail, the next build with more room), then A again.  Every build, timed and
    replayed, equals its oracle (DBIndexer.java:237-405)."""
    a = fasta.config("human").slice(0, 3000)
    spike = a.residues.copy()
    e = int(a.offsets[1500])
    spike[:e] = np.resize(np.frombuffer(b"GAAAAAAK", np.uint8), e)
    b = fasta.PackedProteins(spike, a.offsets.copy(), a.defs)
    cp = DBIndexSearchParams.semi_tryptic(2).to_c()
    oa, ob = cref.Index(cp, a.residues, a.offsets), cref.Index(cp, b.residues, b.offsets)
    with Engine(cp) as eng:
        seen_redo = False
        for k, (p, o) in enumerate([(a, oa), (a, oa), (a, oa), (b, ob), (b, ob), (b, ob), (a, oa), (a, oa)]):
            eng.build(p)
            names = _stages(eng)
            assert_index_equal(eng, o, f"semi build {k}")
            if k in (1, 2):
                assert {"part_hist", "bin_scatter"} <= names, (k, names)
            if k == 3:  # A's region capacities: the spike overflows one, the radix tail redoes it
                seen_redo = "bin_scatter" not in names and "radix_scatter" in names
        assert seen_redo, "the spike did not overflow a region"
        eng.set_timing(False)
        for k in range(3):
            eng.build(a)
            assert_index_equal(eng, oa, f"semi untimed {k}")
        m, t = query_masses(oa, 3000, seed=5)
        assert_queries_equal(eng, oa, m, t, "semi queries")


def _dense_block(rng, n_res):
    """Residues with a K/R every 7-9 positions (random other residues between):
    every cleavage-site start has maxMC + 1 candidate ends past MIN_PEP_LENGTH,
    ~1 500 record slots per 4096-start digest tile -- above the LDS stage."""
    other = np.frombuffer(b"ACDEFGHILMNQSTVWY", np.uint8)
    out, n = [], 0
    while n < n_res:
        k = int(rng.integers(6, 9))
        seg = other[rng.integers(0, len(other), k)]
        out.append(np.append(seg, np.frombuffer(b"KR", np.uint8)[rng.integers(0, 2)]))
        n += k + 1
    return np.concatenate(out)[:n_res]


@pytest.mark.parametrize("part_stage", [1, 0])
def test_part_stage_paths(Engine, part_stage):
    """The partitioning digest keeps a tile's records in LDS (12 B each: mass,
    candidate index and length; tag, protein and offset rebuilt from the
    window) when its slot bound fits, else writes them through HBM slots
    (option part_stage=0: every tile).  One proteome holds both kinds of
    tile -- a block of cleavage-dense proteins (~1 500 slots a tile) and
    ordinary ones -- plus walks past the 128-position horizon (glycine runs
    under a 20000-Da maxMH: walk_global into the stage) and empty / short
    proteins; cold, warm timed and replayed builds equal the oracle
    (DBIndexer.java:237-405)."""
    rng = np.random.default_rng(21)
    base = fasta.config("human").slice(0, 9000)
    seqs = base.sequences()
    dense = _dense_block(rng, 300_000).tobytes().decode()
    cut = [0] + sorted(int(x) for x in rng.integers(1, len(dense), 700)) + [len(dense)]
    seqs[2000:2000] = [dense[a:b] for a, b in zip(cut[:-1], cut[1:])]
    longw = ["G" * 150 + "K" + "AAAAAAR", "M" + "G" * 140 + "R" + "GGGGGGGK", "GGGGGGK" + "G" * 200,
             "A" * 129 + "KR" + "G" * 131, "PEPTIDEK" + "G" * 300 + "K", "", "K", "GGGGK"]
    for i, s in enumerate(longw * 20):
        seqs.insert(5000 + 37 * i, s)
    pp = fasta.PackedProteins.from_sequences(seqs, [fasta.uniprot_header(i) for i in range(len(seqs))])
    cp = DBIndexSearchParams.trypsin(2, max_precursor_mass=20000.0).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    with Engine(cp, options={"part_stage": part_stage}) as eng:
        for k in range(4):
            eng.build(pp)
            if k >= 2:
                assert "bin_scatter" in _stages(eng), (k, _stages(eng))
            assert_index_equal(eng, oix, f"part_stage={part_stage} build {k}")
        eng.set_timing(False)
        for k in range(3):
            eng.build(pp)
            assert_index_equal(eng, oix, f"part_stage={part_stage} replay {k}")
        m, t = query_masses(oix, 4000, seed=17)
        assert_queries_equal(eng, oix, m, t, "queries")


def test_part_stage_long_protein(Engine):
    """A protein of 2^20 + 300 residues: record lengths may not fit the LDS
    stage's 20 bits, so every tile takes the HBM slots; the index equals the
    oracle (the record layout: 2 x 21 bits + the protein id)."""
    rng = np.random.default_rng(5)
    base = fasta.config("human").slice(0, 4000)
    seqs = base.sequences()
    other = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
    seqs.insert(1000, other[rng.integers(0, 20, (1 << 20) + 300)].tobytes().decode())
    pp = fasta.PackedProteins.from_sequences(seqs, [fasta.uniprot_header(i) for i in range(len(seqs))])
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    with Engine(cp) as eng:
        for k in range(3):
            eng.build(pp)
            assert_index_equal(eng, oix, f"long protein build {k}")
        assert "bin_scatter" in _stages(eng)
