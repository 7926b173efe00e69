"""GPU: the N-rank RCCL driver (dbi_build_sharded, dbi_query_sharded,
dbi_shard_replicate) run by N PROCESSES on one GPU.  RCCL refuses two ranks
on one device, so the communicator is the host-staged test transport
(dbi_comm_init_host: the same collectives through POSIX shared memory); every
other line of the driver is the production one: the owner split reused by warm
builds and its hash in the count matrix, the sampled split with the
cost-profile fingerprint, failure agreement, the exchange, the owner merge
whose counters come back with the totals all-gather, the replica and the
routed queries.  Every build's owner slices, concatenated in rank order, must
equal the oracle's index of the whole proteome (VERDICT r03 weak item 6;
ADVICE r03: ranks whose splits differ must not split the index).

Reference: the one-thread build DBIndexer.run (DBIndexer.java:508-684) and
IndexMerge.getMergedData (DBIndexStoreSQLiteByteIndexMerge.java:620-719)."""
from __future__ import annotations

import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NPROT = 600


def _rank_main(world: int, rank: int, name: str, plan: dict, q) -> None:
    import traceback
    try:
        from dbindex_amd import fasta, shard
        from dbindex_amd._native import DBIndexStoreException, DeviceBuffer, synchronize
        from dbindex_amd.engine import Engine
        from dbindex_amd.params import DBIndexSearchParams
        pp = fasta.config(plan.get("config", "1k")).slice(0, plan.get("nprot", NPROT))
        cp = DBIndexSearchParams.trypsin(2).to_c()
        d_res = DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), 0)
        d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), 0)
        synchronize(0)
        comm = shard.ShardComm.host(name, world, rank, 0, 16 << 20)
        b, e = shard.protein_ranges(pp.offsets, world)[rank]
        out = {"builds": []}
        eng = Engine(cp, 0)
        try:
            eng.set_timing(False)
            for k in range(plan["builds"]):
                if plan.get("reopen", {}).get(k) == rank:  # a fresh handle: no split, no cost profile
                    eng.close()
                    eng = Engine(cp, 0)
                    eng.set_timing(False)
                kind = plan.get("mutate", {}).get(k)
                if kind:  # new contents in the same device buffers (same pointers and sizes)
                    res2, off2 = _mutated(pp, kind)
                    d_res.upload(np.concatenate([res2, np.zeros(16, np.uint8)]))
                    d_off.upload(off2.astype(np.uint64))
                    synchronize(0)
                opts = plan.get("options", {}).get(k, {})  # {name: (value, value after the build)}
                for key, (val, _) in opts.items():
                    eng.set_option(key, val)
                try:
                    st = shard.build_sharded(eng, comm, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, b, e)
                    out["builds"].append(dict(ok=True, export=eng.export(), sampled=st.split_sampled,
                                              rounds=st.split_rounds, g_total=st.g_total, g_unique=st.g_unique,
                                              g_keys=st.g_keys, key_lo=st.key_lo, key_hi=st.key_hi,
                                              stages=sorted({n for n, _, _ in eng.stage_times()})))
                except DBIndexStoreException as ex:
                    out["builds"].append(dict(ok=False, error=str(ex)))
                for key, (_, after) in opts.items():
                    eng.set_option(key, after)
            if plan.get("queries"):
                rng = np.random.Generator(np.random.PCG64(100 + rank))
                m = rng.uniform(500.0, 3000.0, 400)
                t = m * 2e-5
                dm, dt = DeviceBuffer.from_numpy(m, 0), DeviceBuffer.from_numpy(t, 0)
                df, dc = DeviceBuffer(8 * m.shape[0], 0), DeviceBuffer(8 * m.shape[0], 0)
                shard.query_sharded(eng, comm, dm.ptr, dt.ptr, m.shape[0], df.ptr, dc.ptr)
                out["routed"] = (m, t, df.download(np.uint64, m.shape[0]), dc.download(np.uint64, m.shape[0]))
                shard.replicate(eng, comm)
                out["replica"] = eng.export()
                out["replica_query"] = eng.query(m, t)
        finally:
            eng.close()
        comm.close()
        q.put((rank, out))
    except Exception:  # the parent reports it
        q.put((rank, {"crash": traceback.format_exc()}))


def _mutated(pp, kind: str):
    """The proteome rewritten in place between builds: 'dense' -- every third
    residue of the first half a K (far more cleavage sites: more digest slots
    than the last build reserved); 'offsets' -- the same residues with every
    inner protein boundary moved three residues on (the shards' residue
    ranges change under the same protein ranges)."""
    res = pp.residues.copy()
    off = pp.offsets.astype(np.int64).copy()
    if kind == "dense":
        res[np.arange(0, int(off[off.shape[0] // 2]), 3)] = ord("K")
    elif kind == "offsets":
        off[1:-1] += 3
        assert np.all(np.diff(off) > 0)
    else:
        raise ValueError(kind)
    return res, off.astype(np.uint64)


HOOK_OPTIONS = ("test_fail", "test_split_skew")


def _run(world: int, plan: dict):
    from dbindex_amd._native import HOOKS_PATH
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = "/dbi_test_" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_rank_main, args=(world, r, name, plan, q)) for r in range(world)]
    # the test hooks live in the test-build library only: the ranks of a plan
    # that sets them load it (a spawned child reads DBI_LIB_PATH at import)
    hooks = any(k in HOOK_OPTIONS for opts in plan.get("options", {}).values() for k in opts)
    saved = os.environ.get("DBI_LIB_PATH")
    if hooks:
        os.environ["DBI_LIB_PATH"] = HOOKS_PATH
    try:
        for p in procs:
            p.start()
    finally:
        if hooks:
            if saved is None:
                os.environ.pop("DBI_LIB_PATH", None)
            else:
                os.environ["DBI_LIB_PATH"] = saved
    res = {}
    try:
        for _ in range(world):
            r, out = q.get(timeout=300)
            res[r] = out
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert "crash" not in res[r], f"rank {r}:\n{res[r]['crash']}"
    return [res[r] for r in range(world)]


@pytest.fixture(scope="module")
def oracle():
    from dbindex_amd import _native, fasta
    from dbindex_amd.params import DBIndexSearchParams
    from oracle import cref
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    pp = fasta.config("1k").slice(0, NPROT)
    return cref.Index(DBIndexSearchParams.trypsin(2).to_c(), pp.residues, pp.offsets)


def _assert_whole_index(parts, oix, ctx):
    from dbindex_amd import shard
    g = shard.concat_exports(parts)
    o = oix.unique()
    assert np.array_equal(g["mass"].view(np.uint64), o["mass"].view(np.uint64)), (ctx, "mass")
    for k in ("prot_id", "offset", "length", "occ_off", "occ_prot"):
        assert np.array_equal(g[k].astype(np.uint64), o[k].astype(np.uint64)), (ctx, k)


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_warm_builds_queries_replica(oracle, world):
    """Build 0 samples (no split yet: a second count-matrix round), builds 1-3
    reuse the split the previous build left (one round); each equals the
    oracle.  Routed queries and the replica on every rank, too."""
    res = _run(world, {"builds": 4, "queries": True})
    for k in range(4):
        builds = [r["builds"][k] for r in res]
        assert all(b["ok"] for b in builds), [b.get("error") for b in builds]
        _assert_whole_index([b["export"] for b in builds], oracle, f"world {world} build {k}")
        assert all(b["g_total"] == oracle.n_total and b["g_unique"] == oracle.n_unique for b in builds)
        assert all(b["g_keys"] == oracle.n_keys for b in builds), "a key row split between two owners"
        assert {b["sampled"] for b in builds} == ({1} if k == 0 else {0}), (k, [b["sampled"] for b in builds])
        assert {b["rounds"] for b in builds} == ({2} if k == 0 else {1})
        # owners' key ranges tile the key space in rank order
        assert builds[0]["key_lo"] == -2**31 and builds[-1]["key_hi"] == 2**31 - 1
        assert all(builds[i]["key_hi"] == builds[i + 1]["key_lo"] for i in range(world - 1))
    for r in res:
        m, t, first, count = r["routed"]
        of, oc = oracle.query_batch(m, t)
        assert np.array_equal(count, oc) and np.array_equal(first[count > 0], of[count > 0])
        _assert_whole_index([r["replica"]], oracle, "replica")
        f2, c2 = r["replica_query"]
        assert np.array_equal(c2, oc) and np.array_equal(f2[c2 > 0], of[c2 > 0])


def test_ranks_disagreeing_split_resamples(oracle):
    """Option test_split_skew = rank 1 at build 2: its reused split differs from
    its peers' (what a reopened handle or another build history gives); the
    hashes in the count matrix disagree, every rank samples, and the index
    still equals the oracle -- no peptide split between two owners."""
    res = _run(3, {"builds": 4, "options": {2: {"test_split_skew": (1, -1)}}})
    for k in range(4):
        builds = [r["builds"][k] for r in res]
        assert all(b["ok"] for b in builds), [b.get("error") for b in builds]
        _assert_whole_index([b["export"] for b in builds], oracle, f"skew build {k}")
        want = 2 if k in (0, 2) else 1
        assert {b["rounds"] for b in builds} == {want}, (k, [b["rounds"] for b in builds])


def test_ranks_reopened_handle_converges(oracle):
    """Rank 1 reopens its handle before build 4: a fresh handle has no split
    and no cost profile, so build 4 samples (two rounds) and the profile
    fingerprints differ; every rank drops its profile then, so build 5 already
    reuses one common split (the ranks used to keep disagreeing,
    build after build, while the reopened rank's fresh profile differed from
    its peers' averaged ones)."""
    res = _run(3, {"builds": 7, "reopen": {4: 1}})
    for k in range(7):
        builds = [r["builds"][k] for r in res]
        assert all(b["ok"] for b in builds), [b.get("error") for b in builds]
        _assert_whole_index([b["export"] for b in builds], oracle, f"reopen build {k}")
        want = 2 if k in (0, 4) else 1
        assert {b["rounds"] for b in builds} == {want}, (k, [b["rounds"] for b in builds])


@pytest.mark.parametrize("phase", ["digest", "partition", "merge"])
def test_ranks_failure_is_agreed(oracle, phase):
    """A local failure on rank 1 (option test_fail = <phase>@1) at build 1: every
    rank returns an error (no rank waits in a collective), and the next build
    of the same handles and communicator equals the oracle."""
    res = _run(2, {"builds": 3, "options": {1: {"test_fail": (phase + "@1", "")}}})
    for r, out in enumerate(res):
        assert out["builds"][0]["ok"] and out["builds"][2]["ok"], (r, out["builds"])
        assert not out["builds"][1]["ok"], (r, phase)
        assert ("injected" in out["builds"][1]["error"]) == (r == 1), (r, out["builds"][1]["error"])
    _assert_whole_index([out["builds"][2]["export"] for out in res], oracle, f"after a {phase} failure")


@pytest.mark.parametrize("kind", ["dense", "offsets"])
def test_ranks_device_sized_digest_redone(oracle, kind):
    """Warm builds digest their shard device-sized (no host round trip before
    the count matrix).  Build 2 rewrites the proteome in place: 'dense' makes
    the digest outgrow the slots the last build reserved, 'offsets' moves the
    shards' residue ranges; either way the device flags it in the count
    matrix, that rank digests again synchronously, every rank gathers again
    (two rounds), and builds 2-3 equal the oracle of the rewritten proteome."""
    from dbindex_amd import fasta
    from dbindex_amd.params import DBIndexSearchParams
    from oracle import cref
    res = _run(2, {"builds": 4, "mutate": {2: kind}})
    pp = fasta.config("1k").slice(0, NPROT)
    r2, o2 = _mutated(pp, kind)
    oix2 = cref.Index(DBIndexSearchParams.trypsin(2).to_c(), r2, o2)
    for k in range(4):
        builds = [r["builds"][k] for r in res]
        assert all(b["ok"] for b in builds), (k, [b.get("error") for b in builds])
        _assert_whole_index([b["export"] for b in builds], oracle if k < 2 else oix2, f"{kind} build {k}")
    assert {b["rounds"] for b in [r["builds"][1] for r in res]} == {1}
    assert {b["rounds"] for b in [r["builds"][2] for r in res]} == {2}, [r["builds"][2]["rounds"] for r in res]


def test_ranks_owner_depth_bins():
    """The RCCL driver's warm owners on depth bins, two
    ranks over 6 000 human-scale proteins: build 0 samples its split (each
    owner's first merge: the radix tail), build 1 reuses it -- the same key
    ranges -- so every owner samples the map from its own previous slice and
    partitions the received records by depth bin; later builds follow the
    cost profile's splits.  Every build equals the oracle."""
    from dbindex_amd import _native, fasta
    from dbindex_amd.params import DBIndexSearchParams
    from oracle import cref
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    pp = fasta.config("human").slice(0, 6000)
    oix = cref.Index(DBIndexSearchParams.trypsin(2).to_c(), pp.residues, pp.offsets)
    res = _run(2, {"builds": 4, "config": "human", "nprot": 6000})
    for k in range(4):
        builds = [r["builds"][k] for r in res]
        assert all(b["ok"] for b in builds), [b.get("error") for b in builds]
        _assert_whole_index([b["export"] for b in builds], oix, f"owner depth build {k}")
        assert all(b["g_total"] == oix.n_total and b["g_unique"] == oix.n_unique for b in builds)
    depth = [["bin_scatter" in b["stages"] for b in r["builds"]] for r in res]
    assert not any(d[0] for d in depth) and all(d[1] for d in depth), depth
