"""GPU parity of the sharded build (dbi_shard_* / dbi_build_sharded): the
owners' unique tables, concatenated in shard order, must equal the oracle's
single-store index of the whole proteome bit for bit, and queries answered by
the owners must equal the oracle's getSequences(m, tol).

Several shards run in one process on one GPU (dbi_shard_exchange_local);
the RCCL driver runs with one rank (a real multi-rank exchange needs one GPU
per rank: bench.py --gpus N).
"""
from __future__ import annotations

import numpy as np
import pytest

from dbindex_amd import fasta, shard
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref
from tests.helpers import query_masses

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from dbindex_amd import _native
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    return _native


def _inputs(native, pp):
    d_res = native.DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), 0)
    d_off = native.DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), 0)
    return d_res, d_off


def _assert_sharded_equal(engines, oix, ctx, nq=1500):
    parts = [e.export() for e in engines]
    g = shard.concat_exports(parts)
    o = oix.unique()
    sts = [shard.shard_stats(e) for e in engines]
    assert sum(s.n_total for s in sts) == oix.n_total, (ctx, "n_total")
    assert sum(s.n_dropped for s in sts) == oix.n_dropped, (ctx, "n_dropped")
    assert sum(s.n_received for s in sts) == oix.n_kept, (ctx, "n_kept")
    assert sum(s.n_unique for s in sts) == oix.n_unique, (ctx, "n_unique")
    assert sum(s.n_keys for s in sts) == oix.n_keys, (ctx, "n_keys")
    assert np.array_equal(g["mass"].view(np.uint64), o["mass"].view(np.uint64)), (ctx, "mass")
    for k in ("prot_id", "offset", "length", "occ_off", "occ_prot"):
        a, b = g[k].astype(np.uint64), o[k].astype(np.uint64)
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0][:5] if a.shape == b.shape else "shape"
            raise AssertionError(f"{ctx}: {k} differs at {bad}")
    keys = np.concatenate([e.entry_keys() for e in engines])
    assert np.array_equal(keys, oix.entry_keys()), (ctx, "entry keys")
    # owner key ranges tile the key line in shard order
    for a, b in zip(sts, sts[1:]):
        assert a.key_hi == b.key_lo, (ctx, "key ranges")
    # queries: every owner answers for its slice; slices are adjacent in the
    # global table, so the union is one contiguous id range
    m, t = query_masses(oix, nq)
    # windows wide enough to meet several owners, and past the last bucket
    m = np.concatenate([m, [3000.0, 1000.0, 5999.0, 7999.0, 600.0]])
    t = np.concatenate([t, [2500.0, 600.0, 0.5, 5.0, 700.0]])
    of, oc = oix.query_batch(m, t)
    first = np.full(m.shape[0], np.iinfo(np.uint64).max, np.uint64)
    count = np.zeros(m.shape[0], np.uint64)
    base = 0
    for e, p in zip(engines, parts):
        f, c = e.query(m, t)
        hit = c > 0
        first[hit] = np.minimum(first[hit], f[hit] + np.uint64(base))
        count += c
        base += p["mass"].shape[0]
    assert np.array_equal(count, oc), (ctx, "query counts")
    hit = oc > 0
    assert np.array_equal(first[hit], of[hit]), (ctx, "query first ids")
    # routed queries: each shard brings its own part of the batch (one shard none)
    k = len(engines)
    cuts = np.linspace(0, m.shape[0], k + 1).astype(int)
    if k > 2:
        cuts[1] = 0
    batches = [(m[a:b], t[a:b]) for a, b in zip(cuts, cuts[1:])]
    res = shard.query_sharded_local(engines, batches)
    rf = np.concatenate([f for f, _ in res])
    rc = np.concatenate([c for _, c in res])
    assert np.array_equal(rc, oc), (ctx, "routed query counts")
    assert np.array_equal(rf[hit], of[hit]), (ctx, "routed query first ids")
    assert np.all(rf[~hit] == 0), (ctx, "routed empty queries")


def _run_local(native, prm, pp, k, ranges=None, ctx=""):
    from dbindex_amd.engine import Engine
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    d_res, d_off = _inputs(native, pp)
    ranges = ranges or shard.protein_ranges(pp.offsets, k)
    engines = [Engine(cp, 0) for _ in range(k)]
    try:
        for rep in ("cold", "warm"):
            shard.build_sharded_local(engines, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, ranges)
            _assert_sharded_equal(engines, oix, f"{ctx} k={k} [{rep}]")
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("k", [1, 2, 3, 5, 8])
def test_sharded_local_tryptic(native, k):
    _run_local(native, DBIndexSearchParams.trypsin(2), fasta.config("1k"), k, ctx="1k tryp2")


@pytest.mark.parametrize("name,prm,nprot,k", [
    ("semi2", DBIndexSearchParams.semi_tryptic(2), 300, 3),
    ("tryp3", DBIndexSearchParams.trypsin(3), 1000, 4),
    ("tryp0", DBIndexSearchParams.trypsin(0), 1000, 2),
    ("nonspec", DBIndexSearchParams.non_specific(50), 60, 4),
    ("mand_K", DBIndexSearchParams.trypsin(2, mandatory_internal_aas="K"), 500, 3),
])
def test_sharded_local_params(native, name, prm, nprot, k):
    _run_local(native, prm, fasta.config("1k").slice(0, nprot), k, ctx=name)


def test_sharded_local_uneven_and_empty_shards(native):
    pp = fasta.config("1k").slice(0, 200)
    # an empty shard, a one-protein shard, and the rest
    ranges = [(0, 0), (0, 1), (1, 150), (150, 150), (150, 200)]
    _run_local(native, DBIndexSearchParams.trypsin(2), pp, 5, ranges=ranges, ctx="uneven")


def test_sharded_local_duplicates_across_shards(native):
    # the same proteins in every shard: every peptide has one owner and its
    # occurrence list spans all shards in protein order
    base = fasta.config("1k").slice(0, 50).sequences()
    pp = fasta.PackedProteins.from_sequences(base * 4)
    _run_local(native, DBIndexSearchParams.trypsin(2), pp, 4, ctx="dups")


def test_sharded_human_scale(native):
    _run_local(native, DBIndexSearchParams.trypsin(2), fasta.config("human"), 4, ctx="human")


@pytest.mark.parametrize("full_path", ["0", "1"])
def test_sharded_rccl_single_rank(native, full_path):
    """One rank: the single-owner build (the single-device build plus the
    shard bookkeeping), and with option shard_full_path=1 the general path
    (samples, partition, exchange to itself, owner merge)."""
    from dbindex_amd.engine import Engine
    pp = fasta.config("1k")
    prm = DBIndexSearchParams.trypsin(2)
    cp = prm.to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    d_res, d_off = _inputs(native, pp)
    comm = shard.ShardComm(shard.ShardComm.unique_id(), 1, 0, 0)
    try:
        with Engine(cp, 0, options={"shard_full_path": int(full_path)}) as eng:
            for rep in ("cold", "warm"):
                st = shard.build_sharded(eng, comm, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins,
                                         0, pp.n_proteins)
                assert st.g_total == oix.n_total and st.g_unique == oix.n_unique and st.g_keys == oix.n_keys
                _assert_sharded_equal([eng], oix, f"rccl x1 [{rep}]")
            # routed queries over RCCL (one rank: the owner is this rank)
            m, t = query_masses(oix, 3000)
            of, oc = oix.query_batch(m, t)
            dm, dt = native.DeviceBuffer.from_numpy(m, 0), native.DeviceBuffer.from_numpy(t, 0)
            df, dc = native.DeviceBuffer(8 * m.shape[0], 0), native.DeviceBuffer(8 * m.shape[0], 0)
            shard.query_sharded(eng, comm, dm.ptr, dt.ptr, m.shape[0], df.ptr, dc.ptr)
            f, c = df.download(np.uint64, m.shape[0]), dc.download(np.uint64, m.shape[0])
            assert np.array_equal(c, oc) and np.array_equal(f[oc > 0], of[oc > 0])
            # all-gatherv of one rank: a copy
            src = native.DeviceBuffer.from_numpy(np.arange(100, dtype=np.uint8), 0)
            dst = native.DeviceBuffer(100, 0)
            comm.allgatherv(src.ptr, dst.ptr, [100])
            assert np.array_equal(dst.download(np.uint8, 100), np.arange(100, dtype=np.uint8))
    finally:
        comm.close()


def test_shard_phase_order(native):
    from dbindex_amd import _native
    from dbindex_amd.engine import Engine
    with Engine(DBIndexSearchParams.trypsin(2).to_c(), 0) as eng:
        with pytest.raises(_native.DBIndexStoreException):
            _native.check(_native.lib().dbi_shard_merge(eng.h))


def _failure_case(phase: str, q) -> None:
    """test_sharded_rccl_local_failure_is_reported's body, in a process that
    loaded the test-hook library (option test_fail exists only there)."""
    import traceback
    try:
        from dbindex_amd import _native as native
        from dbindex_amd.engine import Engine
        pp = fasta.config("1k").slice(0, 200)
        cp = DBIndexSearchParams.trypsin(2).to_c()
        oix = cref.Index(cp, pp.residues, pp.offsets)
        d_res, d_off = _inputs(native, pp)
        m, t = query_masses(oix, 500)
        dm, dt = native.DeviceBuffer.from_numpy(m, 0), native.DeviceBuffer.from_numpy(t, 0)
        df, dc = native.DeviceBuffer(8 * m.shape[0], 0), native.DeviceBuffer(8 * m.shape[0], 0)
        comm = shard.ShardComm(shard.ShardComm.unique_id(), 1, 0, 0)
        try:
            with Engine(cp, 0, options={"shard_full_path": 1}) as eng:  # one rank: the general path
                build = lambda: shard.build_sharded(eng, comm, d_res.ptr, pp.n_residues, d_off.ptr,  # noqa: E731
                                                    pp.n_proteins, 0, pp.n_proteins)
                query = lambda: shard.query_sharded(eng, comm, dm.ptr, dt.ptr, m.shape[0], df.ptr, dc.ptr)  # noqa: E731
                if phase.startswith("q"):
                    build()
                eng.set_option("test_fail", f"{phase}@0")
                try:
                    query() if phase.startswith("q") else build()
                    raise AssertionError("the injected failure was not reported")
                except native.DBIndexStoreException as ex:
                    assert "injected failure" in str(ex), str(ex)
                eng.set_option("test_fail", "")
                st = build()
                assert st.g_total == oix.n_total and st.g_unique == oix.n_unique
                query()
                of, oc = oix.query_batch(m, t)
                f, c = df.download(np.uint64, m.shape[0]), dc.download(np.uint64, m.shape[0])
                assert np.array_equal(c, oc) and np.array_equal(f[oc > 0], of[oc > 0])
        finally:
            comm.close()
        q.put("ok")
    except Exception:
        q.put(traceback.format_exc())


@pytest.mark.parametrize("phase", ["digest", "partition", "buffers", "merge", "qroute", "qbuffers"])
def test_sharded_rccl_local_failure_is_reported(native, phase):
    """A rank that fails locally still joins the next collective with its
    status, so every rank returns an error instead of waiting in RCCL
    (option test_fail injects the failure -- test-build library only,
    libdbindex_hip_hooks.so, in a process of its own; one rank here, the
    agreement collectives are the same at N ranks).  The engine and the
    communicator stay usable: the next build and query batch succeed.  The
    product library does not know the option."""
    import multiprocessing as mp
    import os
    from dbindex_amd.engine import Engine
    with Engine(DBIndexSearchParams.trypsin(2).to_c(), 0) as eng:
        with pytest.raises(native.DBIndexStoreException, match="INVALID"):
            eng.set_option("test_fail", f"{phase}@0")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_failure_case, args=(phase, q))
    saved = os.environ.get("DBI_LIB_PATH")
    os.environ["DBI_LIB_PATH"] = native.HOOKS_PATH
    try:
        p.start()
    finally:
        if saved is None:
            os.environ.pop("DBI_LIB_PATH", None)
        else:
            os.environ["DBI_LIB_PATH"] = saved
    try:
        res = q.get(timeout=240)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert res == "ok", res


@pytest.mark.parametrize("k,nprot", [(1, 300), (3, 1000), (5, 1000)])
def test_replicated_index_local(native, k, nprot):
    """North star's all-gatherv: after a sharded build, every shard's handle
    receives every owner's slice (dbi_shard_replicate_local) and then IS the
    single-device index of the whole proteome: the oracle's index bit for bit,
    and local queries (range lookup and materialised hits) answer for it."""
    from dbindex_amd.engine import Engine
    from tests.helpers import assert_index_equal, assert_queries_equal
    pp = fasta.config("1k").slice(0, nprot)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    d_res, d_off = _inputs(native, pp)
    engines = [Engine(cp, 0) for _ in range(k)]
    try:
        for rep in ("cold", "warm"):
            shard.build_sharded_local(engines, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins,
                                      shard.protein_ranges(pp.offsets, k))
            shard.replicate_local(engines)
            m, t = query_masses(oix, 800)
            for r, e in enumerate(engines):
                assert_index_equal(e, oix, f"replica {r}/{k} [{rep}]")
                assert_queries_equal(e, oix, m, t, f"replica {r}/{k} [{rep}]")
            h = engines[-1].query_hits(m[:50], t[:50])
            o = oix.unique()
            for i in range(50):
                exp = oix.query(float(m[i]), float(t[i]))
                assert np.array_equal(h["ids"][h["row"][i]:h["row"][i + 1]].astype(np.uint64), exp)
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("full_path", ["0", "1"])
def test_replicated_index_rccl_single_rank(native, full_path):
    from dbindex_amd.engine import Engine
    from tests.helpers import assert_index_equal, assert_queries_equal
    pp = fasta.config("1k")
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oix = cref.Index(cp, pp.residues, pp.offsets)
    d_res, d_off = _inputs(native, pp)
    comm = shard.ShardComm(shard.ShardComm.unique_id(), 1, 0, 0)
    try:
        with Engine(cp, 0, options={"shard_full_path": int(full_path)}) as eng:
            for rep in ("cold", "warm"):
                shard.build_sharded(eng, comm, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, 0, pp.n_proteins)
                shard.replicate(eng, comm)
                assert_index_equal(eng, oix, f"rccl replica [{rep}]")
                m, t = query_masses(oix, 1000)
                assert_queries_equal(eng, oix, m, t, f"rccl replica [{rep}]")
    finally:
        comm.close()


def test_bucket_counts_rccl_allreduce_single_rank(native):
    """TrEMBL-style per-bucket counts (dbi_count_buckets) of two protein ranges
    of one proteome, summed by dbi_comm_allreduce_u64 (ncclAllReduce, one
    rank), equal the oracle's buckets of the whole proteome."""
    from dbindex_amd.engine import Engine
    pp = fasta.config("1k").slice(0, 400)
    cp = DBIndexSearchParams.non_specific(30).to_c()
    want = cref.count_buckets(cp, pp.residues, pp.offsets)
    nb = cp.index_factor
    d_hist = native.DeviceBuffer.from_numpy(np.zeros(nb + 1, np.uint64))
    d_sum = native.DeviceBuffer.from_numpy(np.zeros(nb + 1, np.uint64))
    comm = shard.ShardComm(shard.ShardComm.unique_id(), 1, 0, 0)
    try:
        with Engine(cp, 0) as eng:
            for a, b in ((0, 150), (150, 400)):
                part = pp.slice(a, b)
                d_res, d_off = _inputs(native, part)
                eng.count_buckets_device(d_res.ptr, part.n_residues, d_off.ptr, part.n_proteins, d_hist.ptr)
        comm.allreduce_u64(d_hist.ptr, d_sum.ptr, nb + 1)
        assert np.array_equal(d_sum.download(np.uint64, nb + 1), want)
    finally:
        comm.close()


@pytest.mark.parametrize("copies", [3000, 9000])
def test_sharded_merge_grids_outgrown(native, copies):
    """Owner merges size their chunk-list grids (and skip the giant pass) from
    the previous merge on the same handle; a proteome with many more big or
    with giant chunks outgrows them (ERR_GRID) and the merge runs again from
    the received words -- equal to the oracle, then the first proteome again."""
    from dbindex_amd.engine import Engine
    prm = DBIndexSearchParams.trypsin(2)
    cp = prm.to_c()
    plain = fasta.config("human").slice(0, 4000)
    base = fasta.config("1k").sequence(5)
    big = fasta.PackedProteins.from_sequences([base] * copies + [fasta.config("1k").sequence(i) for i in range(6, 40)])
    engines = [Engine(cp, 0) for _ in range(3)]
    try:
        for name, pp in (("plain", plain), (f"x{copies}", big), ("plain again", plain)):
            oix = cref.Index(cp, pp.residues, pp.offsets)
            d_res, d_off = _inputs(native, pp)
            shard.build_sharded_local(engines, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins,
                                      shard.protein_ranges(pp.offsets, 3))
            _assert_sharded_equal(engines, oix, f"merge grids: {name}")
    finally:
        for e in engines:
            e.close()


def test_sharded_cost_profile_splitters(native):
    """Splitters balanced by the merge-cost profile a handle keeps (updated
    by every build, as dbi_build_sharded does) or by an arbitrary skewed one
    move the owner key ranges; the index, the queries and the routed queries
    stay the oracle's."""
    from dbindex_amd.engine import Engine
    prm = DBIndexSearchParams.trypsin(2)
    cp = prm.to_c()
    pp = fasta.config("human").slice(0, 6000)
    oix = cref.Index(cp, pp.residues, pp.offsets)
    d_res, d_off = _inputs(native, pp)
    ranges = shard.protein_ranges(pp.offsets, 4)
    engines = [Engine(cp, 0) for _ in range(4)]
    try:
        sp0 = None
        for rep in range(3):
            sp = shard.build_sharded_local(engines, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, ranges,
                                           balance=True)
            sp0 = sp if sp0 is None else sp0
            _assert_sharded_equal(engines, oix, f"profile: measured merge cost [{rep}]")
            assert all(shard.shard_stats(e).merge_gpu_ms > 0 for e in engines) or rep == 0  # (first: untimed)
        sp2 = shard.build_sharded_local(engines, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, ranges,
                                        profile=(sp0, np.array([20.0, 1.0, 1.0, 5.0])))
        assert sp2[0] < sp0[0]
        _assert_sharded_equal(engines, oix, "profile: skewed")
    finally:
        for e in engines:
            e.close()


def test_split_search_stops_at_the_best_split(native):
    """The cost profile remembers the split whose slowest owner merge was the
    fastest (dbi_shard_cost_update); after three re-splits that do not beat it
    by 2 %, dbi_shard_splitters_profiled returns that split whatever the
    profile says -- the same rule dbi_build_sharded applies to its warm split.
    Then eight real sharded builds, balance on: every one equals the oracle."""
    import ctypes
    from dbindex_amd._native import SHARD_SAMPLES, check, lib
    from dbindex_amd.engine import Engine
    cp = DBIndexSearchParams.trypsin(2).to_c()
    n = 4
    f = cp.mass_group_factor
    masses = np.linspace(600.0, 5000.0, SHARD_SAMPLES)
    samples = np.concatenate([np.concatenate([masses, [1.0]]) for _ in range(n)]).astype(np.float64)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    recs = np.full(n, 1000, np.uint64)
    with Engine(cp, 0) as eng:
        L = lib()

        def profiled():
            out = np.zeros(n, np.int32)
            check(L.dbi_shard_splitters_profiled(eng.h, p(samples), n, p(out)))
            return out[: n - 1].copy()

        best = np.array([int(1500 * f), int(2500 * f), int(3500 * f)], np.int32)
        splits = [best, best + 10, best + 20, best + 30]
        times = [[1.0, 1.0, 1.0, 1.0], [2.0, 1.0, 1.0, 1.0], [1.0, 1.9, 1.0, 1.0], [1.0, 1.0, 3.0, 1.0]]
        for sp, ms in zip(splits, times):
            sp_full = np.concatenate([sp, [0]]).astype(np.int32)
            check(L.dbi_shard_cost_update(eng.h, n, p(sp_full), p(np.array(ms, np.float64)), p(recs)))
        assert np.array_equal(profiled(), best)  # three re-splits no faster: the best split, kept
        # the best split measured again (slower this time) does not restart the search
        check(L.dbi_shard_cost_update(eng.h, n, p(np.concatenate([best, [0]]).astype(np.int32)),
                                      p(np.array([1.5, 1.0, 1.0, 1.0], np.float64)), p(recs)))
        assert np.array_equal(profiled(), best)

        def search(recs_now, splits_ms):
            for sp, ms in splits_ms:
                check(L.dbi_shard_cost_update(eng.h, n, p(np.concatenate([sp, [0]]).astype(np.int32)),
                                              p(np.array(ms, np.float64)), p(recs_now)))

        # the freeze has ways out.  A frozen search only ever runs
        # the best split again; measured far slower (> 2x) the search
        # resumes (the profile's split, not the old best) ...
        search(recs, [(best, [3.0, 1.0, 1.0, 1.0])])
        assert not np.array_equal(profiled(), best)
        # ... and settles again: a faster split, three re-splits no faster
        other = best + 40
        slow = [9.0, 1.0, 1.0, 1.0]
        search(recs, [(other, [1.0, 1.0, 1.0, 1.2]), (best + 50, slow), (best + 60, slow), (best + 70, slow)])
        assert np.array_equal(profiled(), other)
        # a proteome of another size (3x the records) forgets the old best split
        search(recs * np.uint64(3), [(other, [1.0, 1.0, 1.0, 1.2])])
        assert not np.array_equal(profiled(), other)
    pp = fasta.config("human").slice(0, 6000)
    oix = cref.Index(cp, pp.residues, pp.offsets)
    d_res, d_off = _inputs(native, pp)
    ranges = shard.protein_ranges(pp.offsets, 4)
    engines = [Engine(cp, 0) for _ in range(4)]
    try:
        for rep in range(8):
            shard.build_sharded_local(engines, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, ranges,
                                      balance=True)
            _assert_sharded_equal(engines, oix, f"split search [{rep}]")
    finally:
        for e in engines:
            e.close()


def test_sharded_local_merge_graph_replays(native):
    """Untimed repeated builds: each owner's merge is enqueued (build 0),
    captured as a hipGraph (build 1, the same merge again) and replayed (builds
    2-4); a different proteome in between (new key: plain again), then the
    first one again.  Every build equals the oracle."""
    from dbindex_amd.engine import Engine
    cp = DBIndexSearchParams.trypsin(2).to_c()
    a, b = fasta.config("1k"), fasta.config("1k").slice(0, 700)
    oa, ob = (cref.Index(cp, p.residues, p.offsets) for p in (a, b))
    bufs = {id(p): _inputs(native, p) for p in (a, b)}
    engines = [Engine(cp, 0) for _ in range(3)]
    try:
        for e in engines:
            e.set_timing(False)
        for k, (p, o) in enumerate([(a, oa)] * 5 + [(b, ob)] * 3 + [(a, oa)] * 3):
            d_res, d_off = bufs[id(p)]
            shard.build_sharded_local(engines, d_res.ptr, p.n_residues, d_off.ptr, p.n_proteins,
                                      shard.protein_ranges(p.offsets, 3))
            _assert_sharded_equal(engines, o, f"merge graph build {k}", nq=300)
            if k in (2, 3, 4):  # replays: the merge time the cost profile is fed comes from events inside the graph
                assert all(shard.shard_stats(e).merge_gpu_ms > 0 for e in engines), \
                    (k, [shard.shard_stats(e).merge_gpu_ms for e in engines])
    finally:
        for e in engines:
            e.close()


def _stage_names(e):
    return {n for n, _, _ in e.stage_times()}


def test_sharded_owner_depth_bins(native):
    """Warm owner merges on depth bins: an owner's first
    merge takes the radix tail (no slice of its own to sample yet), and so does
    one whose key range moved since its slice (a new split); the next ones
    (the cold build's split reused) partition the received records by depth bin on their way in (the map
    sampled from the owner's previous slice, then reused), enqueued, captured
    as a graph and replayed -- each equal to the oracle; option owner_depth=0
    takes the radix tail again.  Then a proteome of another mass distribution
    under the map of the first: any monotone map gives the exact index (a
    region that overflows is redone by the radix tail), and the first again."""
    from dbindex_amd.engine import Engine
    cp = DBIndexSearchParams.trypsin(2).to_c()
    a = fasta.config("human")
    heavy = str.maketrans({"G": "W", "A": "Y", "S": "F", "V": "H"})
    b = fasta.PackedProteins.from_sequences([s.translate(heavy) for s in a.sequences()])
    oa, ob = (cref.Index(cp, p.residues, p.offsets) for p in (a, b))
    bufs = {id(p): _inputs(native, p) for p in (a, b)}
    engines = [Engine(cp, 0) for _ in range(4)]
    depth_stages = {"part_plan", "bin_scatter"}
    try:
        plan = [(a, oa, "cold")] + [(a, oa, "warm")] * 5 + [(a, oa, "radix")] + [(b, ob, "other")] * 2 + \
               [(a, oa, "back")] * 2
        split = None
        for k, (p, o, what) in enumerate(plan):
            for e in engines:
                e.set_option("owner_depth", 0 if what == "radix" else 1)
                e.set_timing(k < 3 or what != "warm")  # builds 3-5: the merge captured, then replayed
            d_res, d_off = bufs[id(p)]
            # the warm builds of the first proteome reuse the cold build's split
            # (as dbi_build_sharded's warm builds do); the other proteome and the
            # return to the first sample theirs
            sp = shard.build_sharded_local(engines, d_res.ptr, p.n_residues, d_off.ptr, p.n_proteins,
                                           shard.protein_ranges(p.offsets, 4),
                                           split=split if what in ("warm", "radix") else None)
            if k == 0:
                split = sp
            _assert_sharded_equal(engines, o, f"owner depth build {k} ({what})", nq=400)
            names = [_stage_names(e) for e in engines]
            if what in ("cold", "radix"):
                assert all(not (depth_stages & s) for s in names), (k, what)
            elif what == "warm":
                assert all(depth_stages <= s for s in names), (k, what, names)
    finally:
        for e in engines:
            e.close()
