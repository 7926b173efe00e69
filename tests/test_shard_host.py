"""CPU tests of the sharded build's host logic (no GPU, nothing launched):
protein ranges, owner splitters (the C-ABI's host-only dbi_shard_splitters),
owner routing, the assembly of the owners' tables — and the whole plan run by
two gloo ranks, each shard's device work stood in for by the oracle, against
the oracle's single-store index of the whole proteome.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from dbindex_amd import fasta, shard
from dbindex_amd._native import SHARD_SAMPLES
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref


def test_protein_ranges_cover_and_balance():
    pp = fasta.config("1k")
    for k in (1, 2, 3, 7, 16):
        rs = shard.protein_ranges(pp.offsets, k)
        assert rs[0][0] == 0 and rs[-1][1] == pp.n_proteins
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        res = [int(pp.offsets[e] - pp.offsets[b]) for b, e in rs]
        longest = int(np.max(np.diff(pp.offsets.astype(np.int64))))
        assert max(res) - min(res) <= 2 * longest + 1, (k, res)
    # more shards than proteins: empty ranges, still a cover
    rs = shard.protein_ranges(np.array([0, 5, 9], np.uint64), 4)
    assert rs[0][0] == 0 and rs[-1][1] == 2 and all(a[1] == b[0] for a, b in zip(rs, rs[1:]))


def _samples_of(blocks):
    return np.stack([shard.host_samples(np.asarray(b, np.float64)) for b in blocks])


def test_splitters_balance_and_determinism():
    rng = np.random.Generator(np.random.PCG64(5))
    blocks = [np.sort(rng.lognormal(7.3, 0.4, n)) for n in (50_000, 20_000, 80_000, 1)]
    s = _samples_of(blocks)
    for k in (2, 3, 4):
        sp = shard.splitters(s[:k], k, 10000)
        assert np.all(np.diff(sp.astype(np.int64)) >= 0)
        assert np.array_equal(sp, shard.splitters(s[:k].copy(), k, 10000))
        allm = np.concatenate(blocks[:k])
        own = shard.owner_of(allm, sp, 10000)
        counts = np.bincount(own, minlength=k)
        assert counts.max() <= 1.1 * allm.shape[0] / k, counts


def test_splitters_cost_profile():
    """dbi_shard_splitters_cost: uniform band costs give the record-balanced
    splitters; a costly band gets fewer records, so that records x cost
    balance across owners (dbi_build_sharded's feedback between builds)."""
    rng = np.random.Generator(np.random.PCG64(6))
    blocks = [np.sort(rng.lognormal(7.3, 0.4, n)) for n in (60_000, 60_000, 60_000, 60_000)]
    s = _samples_of(blocks)
    k, f = 4, 10000
    sp = shard.splitters(s, k, f)
    assert np.array_equal(shard.splitters(s, k, f, profile=(sp, np.full(k, 2.5))), sp)
    assert np.array_equal(shard.splitters(s, k, f, profile=(np.zeros(0, np.int32), np.full(1, 3.0))), sp)
    cost = np.array([3.0, 1.0, 1.0, 1.0])
    sp2 = shard.splitters(s, k, f, profile=(sp, cost))
    assert sp2[0] < sp[0] and np.all(np.diff(sp2.astype(np.int64)) >= 0)
    allm = np.concatenate(blocks)
    band = shard.owner_of(allm, sp, f)
    own = shard.owner_of(allm, sp2, f)
    load = np.bincount(own, weights=cost[band], minlength=k)
    assert load.max() <= 1.1 * load.sum() / k, load
    assert np.array_equal(sp2, shard.splitters(s, k, f, profile=(sp, cost)))  # deterministic
    with pytest.raises(Exception, match="band costs"):
        shard.splitters(s, k, f, profile=(sp, np.array([1.0, 0.0, 1.0, 1.0])))


def test_splitters_edge_cases():
    # no records anywhere: every key belongs to owner 0
    empty = _samples_of([[], []])
    assert np.all(shard.splitters(empty, 2, 10000) == np.iinfo(np.int32).max)
    # NaN samples (sentinel slots) are skipped, one mass only -> nobody splits it
    s = _samples_of([[1000.0] * 10, [], []])
    s[0, :100] = np.nan
    sp = shard.splitters(s, 3, 10000)
    own = shard.owner_of(np.array([1000.0]), sp, 10000)
    assert own.shape == (1,)
    # the same key never straddles owners
    keys = shard.java_key(np.array([999.99991, 999.99999, 1000.0]), 10000)
    assert keys[0] == keys[1] == 9999999


def test_concat_exports_offsets():
    a = dict(mass=np.array([1.0, 2.0]), prot_id=np.array([0, 1], np.uint32), offset=np.zeros(2, np.uint32),
             length=np.ones(2, np.uint32), occ_off=np.array([0, 2, 3], np.uint64),
             occ_prot=np.array([0, 4, 1], np.uint32))
    b = dict(mass=np.array([3.0]), prot_id=np.array([2], np.uint32), offset=np.zeros(1, np.uint32),
             length=np.ones(1, np.uint32), occ_off=np.array([0, 2], np.uint64), occ_prot=np.array([2, 3], np.uint32))
    g = shard.concat_exports([a, b])
    assert g["occ_off"].tolist() == [0, 2, 3, 5]
    assert g["occ_prot"].tolist() == [0, 4, 1, 2, 3]


# ---- two gloo ranks: the sharded plan end to end, oracle as each shard's engine ----

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank: int, world: int, port: int, cfg: str, nprot: int, missed: int, semi: bool):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pp = fasta.config(cfg).slice(0, nprot)
        prm = DBIndexSearchParams.semi_tryptic(missed) if semi else DBIndexSearchParams.trypsin(missed)
        cp = prm.to_c()
        factor = cp.mass_group_factor
        b, e = shard.protein_ranges(pp.offsets, world)[rank]
        # 1. this shard's digest (oracle stands in for dbi_shard_digest)
        loc = pp.slice(b, e)
        dg = cref.digest(cp, loc.residues, loc.offsets)
        keep = dg.dropped == 0
        n_total, n_dropped = dg.mass.shape[0], int((~keep).sum())
        recs = (dg.mass[keep], dg.pid[keep] + np.uint32(b), dg.offset[keep], dg.length[keep])
        # 2. samples of every shard -> splitters (the product's host function)
        mine = torch.from_numpy(shard.host_samples(recs[0]))
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        split = shard.splitters(np.stack([t.numpy() for t in allv]), world, factor)
        # 3. route to owners (stable) and exchange
        own = shard.owner_of(recs[0], split, factor)
        out = [tuple(a[own == j] for a in recs) for j in range(world)]
        got = [None] * world
        dist.all_gather_object(got, out)
        recv = [np.concatenate([got[i][rank][f] for i in range(world)]) for f in range(4)]
        # 4. owner merge over the whole proteome (oracle stands in for dbi_shard_merge)
        oix = cref.Index(cp, pp.residues, pp.offsets, occurrences=recv)
        part = oix.unique()
        keys = oix.entry_keys()
        sums = torch.tensor([n_total, n_dropped, oix.n_unique, oix.n_keys], dtype=torch.int64)
        dist.all_reduce(sums)
        # 5. replicated index (dbi_shard_replicate): every owner's slice on
        # every rank, which then holds the whole index and answers locally
        parts = [None] * world
        dist.all_gather_object(parts, (part, keys))
        ref = cref.Index(cp, pp.residues, pp.offsets)
        g = shard.concat_exports([p for p, _ in parts])
        o = ref.unique()
        assert sums.tolist() == [ref.n_total, ref.n_dropped, ref.n_unique, ref.n_keys]
        assert np.array_equal(g["mass"].view(np.uint64), o["mass"].view(np.uint64))
        for k in ("prot_id", "offset", "length", "occ_off", "occ_prot"):
            assert np.array_equal(g[k].astype(np.uint64), o[k].astype(np.uint64)), k
        assert np.array_equal(np.concatenate([k for _, k in parts]), ref.entry_keys())
        # this rank's own query batch, answered on its replica alone: a window's
        # hits are the replica rows with lo <= mass <= hi (both ends inclusive)
        rng = np.random.Generator(np.random.PCG64(17 + rank))
        m = g["mass"][rng.integers(0, g["mass"].shape[0], 300)] * (1 + rng.normal(0, 5e-6, 300))
        tol = m * (1 - 1 / (20.0 / 1e6 + 1))
        of, oc = ref.query_batch(m, tol)
        lo = np.searchsorted(g["mass"], m - tol, side="left")
        hi = np.searchsorted(g["mass"], m + tol, side="right")
        assert np.array_equal((hi - lo).astype(np.uint64), oc)
        assert np.array_equal(lo[oc > 0].astype(np.uint64), of[oc > 0])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,cfg,nprot,missed,semi", [(2, "1k", 1000, 2, False), (2, "1k", 200, 2, True),
                                                        (3, "1k", 600, 1, False)])
def test_gloo_strong_split_plan_matches_single_store(world, cfg, nprot, missed, semi):
    """One proteome split by residues over `world` gloo ranks (bench.py
    --scaling strong), owner exchange, owner merge, then the replicated index
    on every rank answering its own queries."""
    import torch.multiprocessing as mp
    mp.spawn(_rank_main, args=(world, _free_port(), cfg, nprot, missed, semi), nprocs=world, join=True)


def _split_restated(samples, k, factor, band_split=None, band_cost=None):
    """dbi_shard_splitters_cost restated: every valid sample's key (int)(m*f)
    weighted by its shard's records per sample x its band's cost; split[j-1] =
    the first key (at a key change) whose preceding weight reaches j/k of the
    total; INT32_MAX when none."""
    ks = []
    for b in samples:
        w = b[-1]
        if not w > 0:
            continue
        for m in b[:-1]:
            if m == m:
                key = int(np.trunc(m * factor))
                c = 1.0
                if band_cost is not None:
                    c = band_cost[int(np.searchsorted(band_split, key, side="right"))]
                ks.append((key, w * c))
    ks.sort(key=lambda x: x[0])
    total = sum(w for _, w in ks)
    out, i, cum = [], 0, 0.0
    for j in range(1, k):
        target = total * j / k
        sp = 2**31 - 1
        while i < len(ks):
            if cum >= target and (i == 0 or ks[i][0] != ks[i - 1][0]):
                sp = ks[i][0]
                break
            cum += ks[i][1]
            i += 1
        out.append(sp)
    return np.array(out, np.int64)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_splitters_match_restatement(seed):
    """The library's sorted-keys + linear quantile walk (sample keys sorted
    once, band costs applied by a moving pointer) equals the weighted-quantile
    definition -- ties of equal keys across shards included (a split lands on
    a key change only)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    k, f = 5, 10000
    # coarse masses: many equal keys across shards
    blocks = [np.sort(np.round(rng.lognormal(7.2, 0.35, n), 2)) for n in (30_000, 9_000, 45_000, 500, 20_000)]
    s = _samples_of(blocks)
    assert np.array_equal(shard.splitters(s, k, f).astype(np.int64), _split_restated(s, k, f))
    band_split = np.sort(rng.integers(5_000_000, 30_000_000, 31)).astype(np.int32)
    band_cost = rng.uniform(0.2, 4.0, 32)
    got = shard.splitters(s, k, f, profile=(band_split, band_cost)).astype(np.int64)
    assert np.array_equal(got, _split_restated(s, k, f, band_split, band_cost))
