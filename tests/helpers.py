"""Shared comparison helpers: the HIP engine vs the oracle (tests only)."""
from __future__ import annotations

import numpy as np

from oracle import cref


def assert_index_equal(eng, oix, ctx: str = "") -> None:
    st = eng.stats()
    assert st.n_total == oix.n_total, (ctx, "n_total", st.n_total, oix.n_total)
    assert st.n_dropped == oix.n_dropped, (ctx, "n_dropped")
    assert st.n_kept == oix.n_kept, (ctx, "n_kept")
    assert st.n_unique == oix.n_unique, (ctx, "n_unique", st.n_unique, oix.n_unique)
    assert st.n_keys == oix.n_keys, (ctx, "n_keys", st.n_keys, oix.n_keys)
    g = eng.export()
    o = oix.unique()
    # masses bit-exact (compare the float64 bit patterns)
    assert np.array_equal(g["mass"].view(np.uint64), o["mass"].view(np.uint64)), (ctx, "mass")
    for k in ("prot_id", "offset", "length", "occ_off", "occ_prot"):
        a, b = g[k], o[k]
        if not np.array_equal(a.astype(np.uint64), b.astype(np.uint64)):
            bad = np.nonzero(a.astype(np.uint64) != b.astype(np.uint64))[0][:5]
            raise AssertionError(f"{ctx}: {k} differs at {bad}: gpu={a[bad]} oracle={b[bad]}")
    assert np.array_equal(eng.entry_keys(), oix.entry_keys()), (ctx, "entry keys")


def query_masses(oix, n: int, seed: int = 7, ppm: float = 20.0):
    """SURVEY.md §8(d) query mix: 90 % indexed masses x (1 + N(0, 5 ppm)),
    10 % uniform on [500, 6000]; tolerance = getToleranceInDalton(m, ppm)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    u = oix.unique()["mass"] if hasattr(oix, "unique") else oix
    k = int(n * 0.9)
    m = np.empty(n, np.float64)
    if u.shape[0]:
        m[:k] = u[rng.integers(0, u.shape[0], k)] * (1 + rng.normal(0, 5e-6, k))
    else:
        m[:k] = rng.uniform(500, 6000, k)
    m[k:] = rng.uniform(500, 6000, n - k)
    tol = m * (1 - 1 / (ppm / 1000000 + 1))
    return m, tol


def assert_queries_equal(eng, oix, masses, tols, ctx: str = "") -> None:
    first, count = eng.query(masses, tols)
    of, oc = oix.query_batch(masses, tols)
    bad = np.nonzero((count != oc) | ((count > 0) & (first != of)))[0]
    assert bad.shape[0] == 0, (ctx, "query mismatch", bad[:5], masses[bad[:5]], first[bad[:5]], of[bad[:5]],
                               count[bad[:5]], oc[bad[:5]])


def tag_collision_proteins():
    """Proteins whose tryptic peptides include isobaric permutations with
    bit-identical fp64 MH+ AND equal 16-bit tag (pairs and a triple), repeated
    in mixed order, so the equal-(mass, tag) groups hold different strings and
    the pinned first-appearance order is exercised."""
    import collections
    import itertools

    from dbindex_amd.params import DBIndexSearchParams, calculate_mass
    from oracle.pyref import peptide_tag

    prm = DBIndexSearchParams.trypsin(0)
    groups = collections.defaultdict(list)
    for perm in itertools.permutations("ACDEFGHM"):
        s = "".join(perm) + "K"
        groups[(np.float64(calculate_mass(s, prm)).view(np.uint64).item(), peptide_tag(s))].append(s)
    pairs = [v for v in groups.values() if len(v) == 2][:40]
    triples = [v for v in groups.values() if len(v) >= 3][:10]
    prots = []
    for a, b in pairs:
        prots.append(b + a + "WWWWWWK" + b)
        prots.append(a + a + b + "GGGGGGGR" + a)
    for t in triples:
        prots.append(t[2] + t[0] + t[1] + t[0])
        prots.append(t[1] * 5 + t[2])
    return prots
