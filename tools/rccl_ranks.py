"""Multi-rank RCCL sharded build: N processes (one rank each, rank r on visible
device r mod #devices), run dbi_build_sharded + dbi_query_sharded + dbi_shard_replicate with
a real N-rank communicator (grouped send/recv, all-gathers, status agreement),
and write their exports for the parent to compare with the oracle.

  python tools/rccl_ranks.py --ranks 2 [--config 1k] [--out DIR]

The parent never touches the GPU (it only spawns the ranks and runs the oracle
on the CPU); the rank-0 worker writes the RCCL unique id to a file the others
poll.  Exit status 0 = every rank's
slice, the concatenated index, routed queries and every replica equal the
oracle's single-store index bit for bit.

Needs one GPU per rank: RCCL 2.27 refuses two ranks on one device at
ncclCommInitRank ("Duplicate GPU detected", invalid usage), measured on the
one-GPU box; there the RCCL path runs with one rank (tests/test_shard_gpu.py)
and N shards exchange by device copies in one process.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

NQ = 4000


def _proteome(config: str, nprot: int):
    from dbindex_amd import fasta
    pp = fasta.config(config)
    return pp.slice(0, nprot) if nprot else pp


def _params(name: str):
    from dbindex_amd.params import DBIndexSearchParams
    return {"tryp2": lambda: DBIndexSearchParams.trypsin(2),
            "semi2": lambda: DBIndexSearchParams.semi_tryptic(2)}[name]()


def _queries(seed: int, rank: int, n: int):
    rng = np.random.default_rng(seed + rank)
    m = rng.uniform(550.0, 5900.0, n)
    t = m * 20e-6
    return m, t


def worker(args) -> int:
    from dbindex_amd import shard
    from dbindex_amd._native import DeviceBuffer, synchronize
    from dbindex_amd.engine import Engine
    rank, n = args.rank, args.ranks
    idf = os.path.join(args.dir, "uid.bin")
    if rank == 0:
        uid = shard.ShardComm.unique_id()
        with open(idf + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(idf + ".tmp", idf)
    else:
        t0 = time.time()
        while not os.path.exists(idf):
            if time.time() - t0 > 60:
                raise RuntimeError("no RCCL unique id from rank 0")
            time.sleep(0.05)
        with open(idf, "rb") as f:
            uid = f.read()
    from dbindex_amd import _native
    dev = rank % max(1, _native.device_count())  # RCCL refuses two ranks on one GPU ("Duplicate GPU detected")
    pp = _proteome(args.config, args.nprot)
    cp = _params(args.params).to_c()
    d_res = DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), dev)
    d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), dev)
    b, e = shard.protein_ranges(pp.offsets, n)[rank]
    comm = shard.ShardComm(uid, n, rank, dev)
    out = {}
    try:
        with Engine(cp, dev) as eng:
            for rep in ("cold", "warm"):
                st = shard.build_sharded(eng, comm, d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins, b, e)
            x = eng.export()
            for k, v in x.items():
                out["slice_" + k] = v
            out["stats"] = np.array([st.g_total, st.g_unique, st.g_keys, st.n_unique], np.uint64)
            # this rank's own query batch, routed to the owners over RCCL
            m, t = _queries(17, rank, NQ)
            dm, dt = DeviceBuffer.from_numpy(m, dev), DeviceBuffer.from_numpy(t, dev)
            df, dc = DeviceBuffer(8 * NQ, dev), DeviceBuffer(8 * NQ, dev)
            shard.query_sharded(eng, comm, dm.ptr, dt.ptr, NQ, df.ptr, dc.ptr)
            out["q_first"], out["q_count"] = df.download(np.uint64, NQ), dc.download(np.uint64, NQ)
            # north_star's replica: every owner's slice onto this rank
            shard.replicate(eng, comm)
            r = eng.export()
            for k, v in r.items():
                out["rep_" + k] = v
            f, c = eng.query(m, t)
            out["rq_first"], out["rq_count"] = f, c
            synchronize(dev)
    finally:
        comm.close()
    np.savez(os.path.join(args.dir, f"rank{rank}.npz"), **out)
    print(f"[rank {rank}] proteins [{b}, {e}) owner slice {x['mass'].shape[0]} uniques", flush=True)
    return 0


def parent(args) -> int:
    from dbindex_amd import shard
    from oracle import cref
    d = args.dir or tempfile.mkdtemp(prefix="dbi_ranks_")
    os.makedirs(d, exist_ok=True)
    uidf = os.path.join(d, "uid.bin")
    if os.path.exists(uidf):
        os.remove(uidf)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", "--rank", str(r),
                               "--ranks", str(args.ranks), "--config", args.config, "--nprot", str(args.nprot),
                               "--params", args.params, "--dir", d], env=env, cwd=ROOT)
             for r in range(args.ranks)]
    rc = 0
    deadline = time.time() + args.timeout
    for p in procs:
        try:
            rc |= p.wait(timeout=max(1.0, deadline - time.time())) != 0
        except subprocess.TimeoutExpired:
            rc = 1
    if rc:
        for p in procs:
            if p.poll() is None:
                p.kill()
        print("a rank failed or timed out", flush=True)
        return 1
    pp = _proteome(args.config, args.nprot)
    oix = cref.Index(_params(args.params).to_c(), pp.residues, pp.offsets)
    o = oix.unique()
    parts = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(args.ranks)]
    whole = shard.concat_exports([{k[6:]: v for k, v in p.items() if k.startswith("slice_")} for p in parts])

    def same(a, b, what):
        for k in ("mass", "prot_id", "offset", "length", "occ_off", "occ_prot"):
            x, y = a[k], b[k]
            if k == "mass":
                x, y = x.view(np.uint64), y.view(np.uint64)
            if x.shape != y.shape or not np.array_equal(x.astype(np.uint64), y.astype(np.uint64)):
                raise AssertionError(f"{what}: {k} differs")

    same(whole, o, "concatenated owner slices")
    for r, p in enumerate(parts):
        g_total, g_unique, g_keys, _ = (int(v) for v in p["stats"])
        assert (g_total, g_unique, g_keys) == (oix.n_total, oix.n_unique, oix.n_keys), f"rank {r} global stats"
        same({k[4:]: v for k, v in p.items() if k.startswith("rep_")}, o, f"replica on rank {r}")
        m, t = _queries(17, r, NQ)
        of, oc = oix.query_batch(m, t)
        hit = oc > 0
        for pre in ("q", "rq"):
            f, c = p[pre + "_first"], p[pre + "_count"]
            assert np.array_equal(c, oc), f"rank {r} {pre} counts"
            assert np.array_equal(f[hit], of[hit]), f"rank {r} {pre} first ids"
    print(f"OK: {args.ranks} RCCL ranks, {args.config}/{args.params} P={pp.n_proteins}: "
          f"{oix.n_unique} uniques, {oix.n_kept} occurrences, owner slices "
          f"{[int(p['slice_mass'].shape[0]) for p in parts]}, replicas and routed queries equal the oracle",
          flush=True)
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--config", default="1k")
    ap.add_argument("--nprot", type=int, default=0)
    ap.add_argument("--params", default="tryp2", choices=("tryp2", "semi2"))
    ap.add_argument("--dir", default="")
    ap.add_argument("--timeout", type=float, default=240.0)
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    return worker(args) if args.worker else parent(args)


if __name__ == "__main__":
    sys.exit(main())
