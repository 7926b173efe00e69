"""GPU parity: the HIP engine (through the C-ABI) vs the oracle on the same
seeded inputs.  Bar: bit-exact for every count, index, id and mass.

Run on an MI355X:  python -m pytest tests -m gpu -x -q
"""
from __future__ import annotations

import numpy as np
import pytest

from dbindex_amd import fasta
from dbindex_amd.params import DBIndexSearchParams, calculate_mass
from oracle import cref
from tests.helpers import assert_index_equal, assert_queries_equal, query_masses, tag_collision_proteins

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine():
    from dbindex_amd.engine import Engine
    from dbindex_amd import _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    return Engine


def _check(Engine, prm, pp, ctx, nq=2000):
    """Build twice on one engine: the first build counts then emits (cold),
    the second runs the fused single-pass digest into the first build's
    capacity (warm).  Both must equal the oracle."""
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    m, t = query_masses(oix, nq)
    with Engine(cp) as eng:
        for phase in ("cold", "warm"):
            eng.build(pp)
            assert_index_equal(eng, oix, f"{ctx} [{phase}]")
            assert_queries_equal(eng, oix, m, t, f"{ctx} [{phase}]")
    return oix


KAT_PROTEINS = [
    "MKWVTFISLLLLFSSAYSRGVFRRDTHKSEIAHRFKDLGEEHFKGLVLIAFSQYLQQCPFDEHVK",  # albumin head
    "PEPTIDEKAAAAAAKPEPTLDEKGGGGGGR",   # I/L isobaric pair inside one protein
    "AAAAAAKPAAAAAAKRPPPPPPRAAAAAAAAA",  # KP / RP (nocut) and a C-terminal non-K/R end
    "PEPTIDEKAAAAAAKPEPTIDEKPEPTIDEK",  # duplicate peptide twice in one protein
    "GGGGGGK",                          # exactly length 7
    "GGGGK",                            # shorter than MIN_PEP_LENGTH
    "",                                 # empty protein
    "K",
    "WWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWWK",  # heavy: crosses maxMH
]


def kat_pack(extra=()):
    seqs = list(KAT_PROTEINS) + list(extra)
    return fasta.PackedProteins.from_sequences(seqs, [fasta.uniprot_header(i) for i in range(len(seqs))])


@pytest.mark.parametrize("name,prm", [
    ("tryp0", DBIndexSearchParams.trypsin(0)),
    ("tryp2", DBIndexSearchParams.trypsin(2)),
    ("tryp2_nocutP", DBIndexSearchParams.trypsin(2, enzyme_nocut_residues="P")),
    ("semi2", DBIndexSearchParams.semi_tryptic(2)),
    ("nonspec", DBIndexSearchParams.non_specific(50)),
    ("mand_K", DBIndexSearchParams.trypsin(2, mandatory_internal_aas="K")),
    ("mand_empty", DBIndexSearchParams.trypsin(2, mandatory_internal_aas="")),
    ("no_h2o", DBIndexSearchParams.trypsin(1, h2o_plus_proton_added=False, min_precursor_mass=100.0)),
    ("terms", DBIndexSearchParams.trypsin(1, cterm=17.0265491, nterm=42.010565)),
])
def test_kat_proteins(Engine, name, prm):
    _check(Engine, prm, kat_pack(), name, nq=500)


@pytest.mark.parametrize("name,prm,nprot", [
    ("1k_tryp0", DBIndexSearchParams.trypsin(0), 1000),
    ("1k_tryp2", DBIndexSearchParams.trypsin(2), 1000),
    ("1k_semi2", DBIndexSearchParams.semi_tryptic(2), 1000),
    ("100_nonspec", DBIndexSearchParams.non_specific(50), 100),
    # params-file static mods: carbamidomethyl C, oxidised M, TMT-like K + N-term
    ("1k_static_mods", DBIndexSearchParams.trypsin(2).with_static_mods(
        {"C": 57.02146, "M": 15.9949, "K": 229.162932}, nterm=229.162932), 1000),
    ("300_semi_n15", DBIndexSearchParams.semi_tryptic(1).with_static_mods({"C": 57.02146}, n15_enrichment=0.98),
     300),
    # warm semi builds: the bounded semi digest (k_digest_semi_bounded), with the bucket drop too
    ("1k_semi0", DBIndexSearchParams.semi_tryptic(0), 1000),
    ("300_semi3", DBIndexSearchParams.semi_tryptic(3), 300),
    ("300_semi_drop", DBIndexSearchParams.semi_tryptic(2, index_factor=7, max_precursor_mass=7999.0), 300),
])
def test_synthetic(Engine, name, prm, nprot):
    pp = fasta.config("1k") if nprot == 1000 else fasta.config("1k").slice(0, nprot)
    _check(Engine, prm, pp, name)


@pytest.mark.parametrize("prm", [DBIndexSearchParams.trypsin(2, max_precursor_mass=20000.0),
                                 DBIndexSearchParams.trypsin(0, max_precursor_mass=20000.0),
                                 DBIndexSearchParams.semi_tryptic(2, max_precursor_mass=20000.0)],
                         ids=["tryp2", "tryp0", "semi2"])
def test_long_light_walks(Engine, prm):
    """Peptides longer than the bounded digests' 128-position horizon: runs of
    glycine (57 Da) without K/R under a 20000-Da maxMH, so a walk finds no
    stop within 128 positions and its mass is still below maxMH there -- it
    goes on from HBM (walk_global) and its slot bound must cover the ends past
    the horizon.  Mixed into the 1k proteome so the second build is warm."""
    long = ["G" * 150 + "K" + "AAAAAAR", "M" + "G" * 140 + "R" + "GGGGGGGK", "GGGGGGK" + "G" * 200,
            "A" * 129 + "KR" + "G" * 131, "PEPTIDEK" + "G" * 300 + "K"]
    base = fasta.config("1k").slice(0, 300)
    seqs = base.sequences()[:150] + long + base.sequences()[150:]
    _check(Engine, prm, fasta.PackedProteins.from_sequences(seqs), "long light walks", nq=500)


@pytest.mark.parametrize("layout", ["short", "empties", "mixed"])
def test_protein_of_start(Engine, layout):
    """The bounded digest finds a start's protein from the start bit map
    (per-word prefix counts) unless two proteins start at one position (empty
    proteins) or more than PST_CAP proteins touch a tile window (then a binary
    search): short proteins (~200 per 4096-residue tile), empty proteins
    between long ones, and both mixed across many tiles, cold and warm."""
    rng = np.random.default_rng({"short": 11, "empties": 12, "mixed": 13}[layout])
    base = fasta.config("1k")
    seqs = []
    for i in range(1500 if layout == "short" else 400):
        s = base.sequence(i % 1000)
        if layout == "short":
            seqs.append(s[: int(rng.integers(4, 30))])
        elif layout == "empties":
            seqs.append(s)
            if i % 25 == 0:  # some tiles hold empty proteins, most do not
                seqs.extend([""] * int(rng.integers(1, 3)))
        else:
            seqs.append(s if i % 2 else s[: int(rng.integers(0, 25))])
    pp = fasta.PackedProteins.from_sequences(seqs, [fasta.uniprot_header(i) for i in range(len(seqs))])
    _check(Engine, DBIndexSearchParams.trypsin(2), pp, f"protein_of {layout}")


@pytest.mark.parametrize("index_factor,maxmh,nprot", [(7, 7999.9, 1000), (3000, 7999.0, 300)])
def test_bucket_drop(Engine, index_factor, maxmh, nprot):
    """BUCKET_MASS_RANGE = 8000 / index_factor (integer division): peptides whose
    bucket exceeds NUM_BUCKETS-1 count in totalSeqCount but are not stored
    (SQLiteMult:277-288); queries touching such buckets return nothing."""
    prm = DBIndexSearchParams.trypsin(4, index_factor=index_factor, max_precursor_mass=maxmh)
    pp = fasta.config("1k").slice(0, nprot)
    oix = _check(Engine, prm, pp, f"drop-{index_factor}")
    assert oix.n_dropped > 0


@pytest.mark.parametrize("copies", [3000, 9000])
def test_big_bins_and_duplicates(Engine, copies):
    """Thousands of copies of one protein: every peptide repeats `copies`
    times, so chunks exceed CHUNK_CAP (3000: 1024-thread LDS bitonic path) or
    BIG_CAP (9000: global-memory path); protein-id lists keep insertion order."""
    base = fasta.config("1k").sequence(5)
    seqs = [base] * copies + [fasta.config("1k").sequence(i) for i in range(6, 40)]
    pp = fasta.PackedProteins.from_sequences(seqs)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    with Engine(cp) as eng:
        st = eng.build(pp)
        assert st.n_big_bins > 0
        assert_index_equal(eng, oix, f"bigbins x{copies}")


@pytest.mark.parametrize("h1", [1, 0])
def test_digest_counted_histogram(Engine, h1):
    """Warm bounded builds of small tails count the first radix pass's
    histogram in the digest (option digest_hist, default on below 16 M slots;
    the radix tail: depth bins off):
    no histogram kernel for that pass, the same index.  ~400 k records: 2^16
    bins, two 8-bit passes, so the LDS counters cover one radix chunk per tile
    and every tile region that crosses a chunk boundary takes the global
    atomic path; cleavage-dense proteins ("AK" repeats: ~8000 slots per
    4096-start tile) span several chunks."""
    base = fasta.config("human")
    seqs = [base.sequence(i) for i in range(4000)]
    seqs[100:100] = ["AK" * 3000, "GAKR" * 1500, "AKK" * 2000]
    pp = fasta.PackedProteins.from_sequences(seqs, [fasta.uniprot_header(i) for i in range(len(seqs))])
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    m, t = query_masses(oix, 1000)
    with Engine(cp, options={"digest_hist": h1, "depth_bins": 0}) as eng:
        hists = []
        for k in range(4):  # cold, warm, warm (captured), replay
            eng.build(pp)
            assert_index_equal(eng, oix, f"digest histogram={h1} [{k}]")
            assert_queries_equal(eng, oix, m, t, f"digest histogram={h1} [{k}]")
            hists.append(sum(1 for n, _, _ in eng.stage_times() if n == "radix_hist"))
    passes = hists[0]  # the cold build: one histogram kernel per radix pass
    assert hists[1] == (passes - 1 if h1 == 1 else passes), hists


@pytest.mark.parametrize("copies", [3000, 9000])
def test_list_grids_outgrown(Engine, copies):
    """Warm builds size the mid / big chunk-list grids from the previous
    build's lists and skip the giant-chunk pass when it had no giant chunks; a
    build with far more big chunks (3000 copies of one protein) or with giant
    ones (9000) than the last one outgrows them (ERR_GRID) and is redone --
    same index as the oracle.  Then the first proteome again."""
    cp = DBIndexSearchParams.trypsin(2).to_c()
    plain = fasta.config("human").slice(0, 12000)
    base = fasta.config("1k").sequence(5)
    seqs = [base] * copies + [fasta.config("1k").sequence(i) for i in range(6, 40)]
    big = fasta.PackedProteins.from_sequences(seqs)
    assert big.residues.size < plain.residues.size  # the second build stays warm (no regrowth)
    o_plain = cref.Index(cp, plain.residues, plain.offsets)
    o_big = cref.Index(cp, big.residues, big.offsets)
    with Engine(cp) as eng:
        st = eng.build(plain)
        assert st.n_big_bins == 0
        assert_index_equal(eng, o_plain, "list grids: plain [cold]")
        st = eng.build(big)
        assert st.n_big_bins > 16
        assert_index_equal(eng, o_big, f"list grids: x{copies} [warm, outgrown]")
        eng.set_timing(True)
        for k in range(3):
            eng.build(plain)
            assert_index_equal(eng, o_plain, f"list grids: plain again [{k}]")
        # the big list was empty in the last build: its kernel is not launched
        # (a build that lists big chunks then is redone, as above)
        st = dict((n, ms) for n, ms, _ in eng.stage_times())
        assert st.get("chunk_sort_big", 0.0) == 0.0 and st["chunk_sort"] > 0.0, st


def _giant_isobaric():
    """~12k proteins whose tryptic peptides are permutations of one
    composition: thousands of bit-identical fp64 masses with different strings
    (one chunk far above BIG_CAP, split on the peptide tag), some repeated."""
    import itertools
    rng = np.random.default_rng(3)
    perms = ["".join(p) for p in itertools.permutations("ACDEFGHM")]
    pick = [perms[i] for i in rng.choice(len(perms), 11000, replace=False)]
    pick += pick[:1500]  # duplicates across proteins
    return [f"MK{p}KWWR" for p in pick]


def _giant_near_isobaric(prm):
    """Peptides with distinct masses packed into a few mDa (residue masses of
    a few letters overridden to tiny values): one mass bin far above BIG_CAP
    holding thousands of different masses (split on the mass bits)."""
    prm.residue_mass.update({"B": 0.0013, "J": 0.00071, "O": 0.000029, "U": 0.0000037, "Z": 0.19})
    rng = np.random.default_rng(5)
    tail = ["".join(rng.choice(list("BJOUZ"), 7)) for _ in range(14000)]
    return [f"MRGGGGGGGGGW{t}K" for t in tail]


def _giant_duplicates():
    """One isobaric spike of ~26k records made of six peptides repeated 3000
    (four of them), 5000 and 9000 times: the split on the tag leaves
    equal-(mass, tag) buckets of 3000 (big leaves of the 512-thread class),
    5000 (the 1024-thread class) and 9000 (above BIG_CAP: the global-memory
    fallback)."""
    import itertools
    perms = ["".join(p) for p in itertools.islice(itertools.permutations("ACDEFGHM"), 0, 40000, 6661)][:6]
    counts = [3000, 3000, 3000, 3000, 5000, 9000]
    return [f"MK{p}KWWR" for p, c in zip(perms, counts) for _ in range(c)]


def _giant_collision():
    """Two different peptides with bit-identical mass AND equal 16-bit tag,
    4 000 + 5 000 + 1 000 occurrences in mixed order: one equal-(mass, tag)
    segment above BIG_CAP holding two strings -- the fallback's LDS path
    finds the collision and hands the segment to the global-memory regroup."""
    import collections
    import itertools
    from dbindex_amd.params import calculate_mass
    from oracle.pyref import peptide_tag
    prm = DBIndexSearchParams.trypsin(0)
    groups = collections.defaultdict(list)
    for perm in itertools.permutations("ACDEFGHM"):
        pep = "".join(perm) + "K"
        groups[(np.float64(calculate_mass(pep, prm)).view(np.uint64).item(), peptide_tag(pep))].append(pep)
        if len(groups[next(reversed(groups))]) == 2:
            break
    a, b = next(v for v in groups.values() if len(v) == 2)
    return [a] * 4000 + [b] * 5000 + [a] * 1000


def _giant_one_peptide():
    """One peptide 17 000 times (beyond the fallback's 16 384-record LDS
    sort: the global-memory path) beside a 9 000-record one (the LDS path)."""
    return ["ACDEFGHMK"] * 17000 + ["MHGFEDCAK"] * 9000


@pytest.mark.parametrize("kind", ["isobaric", "near_isobaric", "duplicates", "collision", "one_peptide"])
def test_giant_chunks(Engine, kind):
    prm = DBIndexSearchParams.trypsin(1)
    seqs = _giant_isobaric() if kind == "isobaric" else _giant_near_isobaric(prm) if kind == "near_isobaric" \
        else _giant_duplicates() if kind == "duplicates" else _giant_collision() if kind == "collision" \
        else _giant_one_peptide()
    pp = fasta.PackedProteins.from_sequences(seqs)
    oix = _check(Engine, prm, pp, f"giant {kind}", nq=800)
    assert oix.n_kept > 8000


@pytest.mark.parametrize("n,dups,copies", [(2600, 0, 300), (3000, 500, 900)])
def test_multi_mass_wide_bins(Engine, n, dups, copies):
    """One mass bin of ~3 000 / ~4 400 records (the big tier's 512- and
    1024-thread classes) holding ~55 distinct fp64 masses within 0.07 mDa (a
    3.7-uDa residue letter repeated 0..19 times, shuffled into one
    composition: ulp-level sums) beside a spike of `copies` repeats of one
    peptide: the semi-tryptic big bins' shape (profiles/r06p2: ~30 masses,
    one dominant) through the block-level compact-key sort; duplicates across
    proteins keep first appearance.  Cold (radix tail) and warm (depth bins)."""
    prm = DBIndexSearchParams.trypsin(0)
    prm.residue_mass.update({"U": 0.0000037})
    rng = np.random.default_rng(9)
    seqs = []
    for _ in range(n):
        core = list("GGAWDEFH") + ["U"] * int(rng.integers(0, 20))
        rng.shuffle(core)
        seqs.append("MR" + "".join(core) + "K")
    seqs += [seqs[int(i)] for i in rng.integers(0, n, dups)]
    seqs[n // 3:n // 3] = ["MRGGUAWDUEFHK"] * copies
    pp = fasta.PackedProteins.from_sequences(seqs)
    oix = _check(Engine, prm, pp, f"multi-mass wide bin {n}+{dups}+{copies}", nq=500)
    assert oix.n_kept == n + dups + copies


def test_isobaric_runs(Engine):
    """I/L swaps give bit-identical masses: equal-mass runs holding several
    peptide strings must group by string, first appearance first."""
    rng = np.random.default_rng(11)
    core = "".join(rng.choice(list("ACDEFGHMNPQSTVWY"), 12))
    seqs = []
    for i in range(400):
        pep = core[:4] + ("I" if rng.random() < 0.5 else "L") + core[5:8] + ("I" if rng.random() < 0.5 else "L") + core[9:]
        seqs.append("MK" + pep + "K" + "".join(rng.choice(list("ACDEFGHMNPQSTVWY"), 20)) + "R")
    pp = fasta.PackedProteins.from_sequences(seqs)
    _check(Engine, DBIndexSearchParams.trypsin(1), pp, "isobaric")


def test_zero_mass_long_walks(Engine):
    """Residues with mass 0 (unknown letters) let a walk run past the LDS halo."""
    prm = DBIndexSearchParams.trypsin(2)
    prm.residue_mass["X"] = 0.0
    seqs = ["AK" + "X" * 700 + "GGGGGGGK" + "X" * 300 + "R", "MKR" + "X" * 5000 + "K"]
    pp = fasta.PackedProteins.from_sequences(seqs + [fasta.config("1k").sequence(1)])
    _check(Engine, prm, pp, "zero-mass")


def test_empty_inputs(Engine):
    prm = DBIndexSearchParams.trypsin(2)
    with Engine(prm) as eng:
        st = eng.build(fasta.PackedProteins.from_sequences([]))
        assert st.n_total == 0 and st.n_unique == 0 and st.n_keys == 0
        f, c = eng.query([1000.0, 2000.0], [0.1, 0.1])
        assert c.sum() == 0
        st = eng.build(fasta.PackedProteins.from_sequences(["", "GGK", ""]))
        assert st.n_total == 0


def test_edge_queries(Engine):
    prm = DBIndexSearchParams.trypsin(2)
    pp = fasta.config("1k").slice(0, 200)
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    u = oix.unique()["mass"]
    qs = [(u[0], 0.0), (u[-1], 0.0), (u[len(u) // 2], 0.0), (999.995, 0.01), (1000.0, 0.0),
          (7999.0, 2.0), (8000.0, 0.0), (3.0, 10.0), (0.0, 0.0), (-5.0, 1.0), (600.0, 1e9),
          (float("nan"), 1.0), (1500.0, float("nan")), (1500.0, -1.0), (u[10], 1e-12),
          (2000.0, float("inf"))]
    m = np.array([q[0] for q in qs])
    t = np.array([q[1] for q in qs])
    with Engine(cp) as eng:
        eng.build(pp)
        assert_queries_equal(eng, oix, m, t, "edge")


def test_exact_mass_lookup(Engine):
    """getProteins(String): IndexUtil.calculateMass + window [m, m] must find
    every indexed peptide (bit-identical masses)."""
    prm = DBIndexSearchParams.trypsin(2)
    pp = fasta.config("1k").slice(0, 300)
    with Engine(prm) as eng:
        eng.build(pp)
        g = eng.export()
        idx = np.linspace(0, g["mass"].shape[0] - 1, 400).astype(np.int64)
        seqs = [pp.sequence(int(g["prot_id"][i]))[int(g["offset"][i]):int(g["offset"][i]) + int(g["length"][i])]
                for i in idx]
        masses = np.array([calculate_mass(s, prm) for s in seqs])
        assert np.array_equal(masses.view(np.uint64), g["mass"][idx].view(np.uint64))
        first, count = eng.query(masses, np.zeros_like(masses))
        assert np.all(count >= 1)
        assert np.all((first <= idx) & (idx < first + count))


def test_rebuild_reuses_workspace(Engine):
    """Workspace reuse across inputs, including a fused (warm) build whose
    output outgrows the previous capacity: the pass is re-run into a grown
    buffer."""
    prm = DBIndexSearchParams.trypsin(2)
    big = fasta.config("1k")
    small = big.slice(0, 50)
    cp = prm.to_c()
    with Engine(cp) as eng:
        eng.build(big)
        eng.build(small)
        assert_index_equal(eng, cref.Index(cp, small.residues, small.offsets), "rebuild-small")
        eng.build(big)
        assert_index_equal(eng, cref.Index(cp, big.residues, big.offsets), "rebuild-big")
    with Engine(cp) as eng:
        eng.build(big.slice(0, 120))      # cold: capacity ~ 120 proteins
        eng.build(big)                    # warm, capacity short -> grown and re-run
        assert_index_equal(eng, cref.Index(cp, big.residues, big.offsets), "outgrow")
        eng.build(big)
        assert_index_equal(eng, cref.Index(cp, big.residues, big.offsets), "outgrow-again")


def test_build_device_pointers(Engine):
    """Residues already resident in HBM (dbi_build_device / dbi_query_device)."""
    from dbindex_amd._native import DeviceBuffer, synchronize
    prm = DBIndexSearchParams.trypsin(2)
    pp = fasta.config("1k")
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    d_res = DeviceBuffer.from_numpy(pp.residues)
    d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64))
    with Engine(cp) as eng:
        eng.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)
        assert_index_equal(eng, oix, "device-ptr")
        m, t = query_masses(oix, 1000)
        dm, dt = DeviceBuffer.from_numpy(m), DeviceBuffer.from_numpy(t)
        df, dc = DeviceBuffer(8 * 1000), DeviceBuffer(8 * 1000)
        eng.query_device(dm.ptr, dt.ptr, 1000, df.ptr, dc.ptr)
        synchronize()
        f, c = eng.query(m, t)
        assert np.array_equal(df.download(np.uint64, 1000), f)
        assert np.array_equal(dc.download(np.uint64, 1000), c)


def test_query_csr_and_peptides(Engine):
    prm = DBIndexSearchParams.trypsin(2)
    pp = fasta.config("1k").slice(0, 300)
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    m, t = query_masses(oix, 300)
    with Engine(cp) as eng:
        eng.build(pp)
        row, ids = eng.query_csr(m, t)
        for i in range(300):
            exp = oix.query(float(m[i]), float(t[i]))
            assert np.array_equal(ids[row[i]:row[i + 1]], exp)
        o = oix.unique()
        sel = np.unique(ids)[:200]
        pep = eng.peptides(sel)
        assert np.array_equal(pep["mass"], o["mass"][sel])
        assert np.array_equal(pep["prot_id"], o["prot_id"][sel])
        assert np.array_equal(pep["occ_begin"], o["occ_off"][sel])
        assert np.array_equal(pep["occ_end"], o["occ_off"][sel + 1])


@pytest.mark.parametrize("copies", [1, 40, 300])
def test_tag_collisions(Engine, copies):
    """Equal (mass, 16-bit tag) groups holding different strings: regrouped by
    first appearance inside the LDS chunk sort (40 copies: big duplicate runs;
    300 copies: equal-mass bins above CHUNK_CAP, the 1024-thread path)."""
    seqs = tag_collision_proteins() * copies
    pp = fasta.PackedProteins.from_sequences(seqs)
    _check(Engine, DBIndexSearchParams.trypsin(0), pp, f"collisions x{copies}", nq=500)
    _check(Engine, DBIndexSearchParams.trypsin(2), pp, f"collisions mc2 x{copies}", nq=500)


@pytest.mark.parametrize("spikes", [(("GGGAAAGGGAK", 600),),
                                    (("GGGAAAGGGAK", 520), ("GGGAAAGGGSK", 530), ("GGGAAAGGGTK", 700))])
def test_tag_collisions_beside_wide_bins(Engine, spikes):
    """A chunk that holds tag-collision groups (regrouped by string in
    k_chunk_sort) AND bins above 512 records, which k_chunk_sort leaves out
    for k_bin_sort_mid (round 4): the left-out ranges must be neither written
    nor counted by the collision path, and their heads come back through the
    mid kernel's add to the chunk's unique count."""
    seqs = list(tag_collision_proteins())
    for pep, n in spikes:  # one tryptic peptide per protein: n identical records
        seqs += [pep] * n
    pp = fasta.PackedProteins.from_sequences(seqs)
    _check(Engine, DBIndexSearchParams.trypsin(0), pp, f"collisions + wide bins {spikes}", nq=300)
    _check(Engine, DBIndexSearchParams.trypsin(2), pp, f"collisions + wide bins mc2 {spikes}", nq=300)


def test_thresholds_on_exact_peptide_masses(Engine):
    """minMH / maxMH set exactly to indexed peptide masses: inclusive bounds
    (DBIndexer.java:284,331) decided on the bit-exact sequential sum, also in
    the cut-stepping count pass (near-threshold starts are recounted exactly)."""
    pp = fasta.config("1k").slice(0, 150)
    d = cref.digest(DBIndexSearchParams.trypsin(2).to_c(), pp.residues, pp.offsets)
    m = np.sort(d.mass)
    for lo, hi in [(m[100], m[-100]), (m[7], m[8]), (np.nextafter(m[50], 0), np.nextafter(m[-50], 1e9))]:
        prm = DBIndexSearchParams.trypsin(2, min_precursor_mass=float(lo), max_precursor_mass=float(hi))
        _check(Engine, prm, pp, f"thresholds {lo} {hi}", nq=300)


@pytest.mark.parametrize("seqs", [
    [],                                    # empty index
    ["PEPTIDEK"],                          # one unique
    ["PEPTIDEK", "PEPTLDEK"],              # two uniques, bit-identical masses
    ["PEPTIDEK", "WWWWWWWWK"],             # two uniques far apart
])
def test_query_directory_edges(Engine, seqs):
    """The query directory (buckets over [first, last] unique mass) brackets
    every bound: queries exactly at, just beside, below and above the uniques,
    zero / huge / infinite tolerances and NaN give the oracle's answer."""
    prm = DBIndexSearchParams.trypsin(0, min_precursor_mass=300.0)
    pp = fasta.PackedProteins.from_sequences(seqs) if seqs else fasta.PackedProteins.from_sequences(["GGK"])
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    u = oix.unique()["mass"]
    base = list(u) + [300.0, 499.9, 5999.0, 7999.0, 1e-3]
    m, t = [], []
    for x in base:
        for dx in (0.0, -1e-9, 1e-9, np.nextafter(x, -np.inf) - x, np.nextafter(x, np.inf) - x):
            for tol in (0.0, 1e-7, 0.5, 3000.0, np.inf):
                m.append(x + dx)
                t.append(tol)
    m += [float("nan"), 900.0, float("inf"), -float("inf")]
    t += [1.0, float("nan"), 1.0, 1.0]
    m, t = np.array(m, np.float64), np.array(t, np.float64)
    with Engine(cp) as eng:
        eng.build(pp)
        assert_queries_equal(eng, oix, m, t, f"dir {len(seqs)}")


def test_size_limits_fail_loudly(Engine):
    """Limits of the 16-B record and the u32 device indices are errors, never
    wrong answers: >= 2^32-1 residues or proteins per device, and a record
    layout of 2 x bits(longest protein) + bits(protein count) > 56."""
    from dbindex_amd import _native
    cp = DBIndexSearchParams.trypsin(2).to_c()
    with Engine(cp) as eng:
        fake = 1 << 20  # never dereferenced: the sizes are rejected first
        with pytest.raises(_native.DBIndexStoreException, match="2\\^32"):
            eng.build_device(fake, (1 << 32) - 1, fake, 10)
        with pytest.raises(_native.DBIndexStoreException, match="2\\^32"):
            eng.build_device(fake, 100, fake, (1 << 32) - 1)
        # longest protein 2^20 residues -> W = 21: at most 2^14 proteins
        long = "AAAAAAK" * ((1 << 20) // 7 + 1)
        seqs = [long] + ["GGGGGGK"] * (1 << 14)
        pp = fasta.PackedProteins.from_sequences(seqs)
        with pytest.raises(_native.DBIndexStoreException, match="56 bits"):
            eng.build(pp)
        ok = fasta.PackedProteins.from_sequences(seqs[:-1])  # 2^14 proteins: fits
        st = eng.build(ok)
        assert st.n_total > 0


def test_concurrent_queries_from_threads(Engine):
    """Query-side calls from several host threads on one handle (ctypes drops
    the GIL): every answer equals the oracle's."""
    import threading
    pp = fasta.config("1k")
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    m, t = query_masses(oix, 4000)
    of, oc = oix.query_batch(m, t)
    errors = []
    with Engine(cp) as eng:
        eng.build(pp)

        def worker(seed):
            rng = np.random.default_rng(seed)
            for _ in range(20):
                sel = rng.integers(0, m.shape[0], 500)
                f, c = eng.query(m[sel], t[sel])
                hit = oc[sel] > 0
                if not (np.array_equal(c, oc[sel]) and np.array_equal(f[hit], of[sel][hit])):
                    errors.append(seed)
                ids = np.unique(rng.integers(0, oix.n_unique, 50)).astype(np.uint64)
                eng.peptides(ids)

        th = [threading.Thread(target=worker, args=(s,)) for s in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    assert not errors


@pytest.mark.parametrize("nprot,nq", [(300, 500), (1000, 3000)])
def test_query_hits_device(Engine, nprot, nq):
    """dbi_query_hits_device: every query's unique ids (getSequences(m, tol),
    DBIndexStoreSQLiteMult.java:315-350) and every hit's protein ids
    (insertion order, duplicates kept, IndexMerge.java:676-681), all
    materialised in HBM, equal the oracle's."""
    prm = DBIndexSearchParams.trypsin(2)
    pp = fasta.config("1k").slice(0, nprot)
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    o = oix.unique()
    m, t = query_masses(oix, nq)
    m[:5] = [float("nan"), 8000.0, -1.0, 0.0, 1e9]  # empty windows
    with Engine(cp) as eng:
        eng.build(pp)
        for _ in range(2):  # second call reuses the grown buffers
            r = eng.query_hits(m, t)
            assert r["row"][0] == 0 and r["occ_row"][0] == 0
            for i in range(nq):
                exp = oix.query(float(m[i]), float(t[i]))
                got = r["ids"][r["row"][i]:r["row"][i + 1]]
                assert np.array_equal(got.astype(np.uint64), exp), i
                prots = r["prot"][r["occ_row"][i]:r["occ_row"][i + 1]]
                want = np.concatenate([o["occ_prot"][o["occ_off"][u]:o["occ_off"][u + 1]] for u in exp]) \
                    if exp.shape[0] else np.zeros(0, np.uint32)
                assert np.array_equal(prots, want), i
                starts = r["hit_occ"][r["row"][i]:r["row"][i + 1]]
                assert np.array_equal(starts.astype(np.uint64), (o["occ_off"][exp] - o["occ_off"][exp[0]])
                                      if exp.shape[0] else np.zeros(0, np.uint64)), i


@pytest.mark.parametrize("name,prm", [
    ("tryp2", DBIndexSearchParams.trypsin(2)),
    ("nonspec", DBIndexSearchParams.non_specific(30)),
    ("semi2", DBIndexSearchParams.semi_tryptic(2)),
    ("mandK", DBIndexSearchParams.trypsin(2, mandatory_internal_aas="K")),
    ("drop", DBIndexSearchParams.trypsin(4, index_factor=7, max_precursor_mass=7999.0)),
    ("drop13", DBIndexSearchParams.trypsin(4, index_factor=13, max_precursor_mass=7999.0)),
    ("fine", DBIndexSearchParams.trypsin(2, index_factor=64)),
    ("nonspec9", DBIndexSearchParams.non_specific(50, index_factor=9)),
    ("fine_nonspec", DBIndexSearchParams.non_specific(40, index_factor=64)),
])
def test_count_buckets(Engine, name, prm):
    """dbi_count_buckets: occurrences per SQLiteMult bucket
    (DBIndexStoreSQLiteMult.java:215-217; last entry: past the last bucket)
    equal the oracle's, by the bit-map count (boundaries by binary search,
    walks where one lies within CUT_EPS) and by the walk (semi / mandatory)."""
    from dbindex_amd._native import DeviceBuffer
    pp = fasta.config("1k").slice(0, 300)
    cp = prm.to_c()
    want = cref.count_buckets(cp, pp.residues, pp.offsets)
    total = cref.count(cp, pp.residues, pp.offsets)
    d_res = DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]))
    d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64))
    d_hist = DeviceBuffer.from_numpy(np.zeros(cp.index_factor + 1, np.uint64))
    with Engine(cp) as eng:
        assert eng.count_buckets_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, d_hist.ptr) == total
    assert np.array_equal(d_hist.download(np.uint64, cp.index_factor + 1), want), name
    if name.startswith("drop"):
        assert want[-1] > 0  # occurrences past the last bucket (SQLiteMult's drops) are counted


def test_count_buckets_rejects_large_index_factor(Engine):
    from dbindex_amd._native import DBIndexStoreException, DeviceBuffer
    pp = fasta.config("1k").slice(0, 10)
    cp = DBIndexSearchParams.trypsin(2, index_factor=100).to_c()
    d_res = DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]))
    d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64))
    d_hist = DeviceBuffer(8 * 101)
    with Engine(cp) as eng:
        with pytest.raises(DBIndexStoreException, match="index_factor"):
            eng.count_buckets_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, d_hist.ptr)
