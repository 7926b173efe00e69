#!/usr/bin/env python3
"""bench.py — peptides indexed/sec on the MI355X engine (BASELINE.json metric).

Step = one full index build (digest -> mass bins -> per-bin sort + dedup ->
unique table + occurrence CSR) over one synthetic proteome already resident in
HBM.  Default workload at N=1: the SwissProt-scale FASTA the metric is quoted
on (BASELINE.json configs[2] "SwissProt (~560k proteins), trypsin, 2 missed
cleavages", which fits one MI355X) as a seeded synthetic proteome (SURVEY.md
§8(d), seed 3).  --config human is configs[1] (20k proteins, seed 2).
N>1 (torchrun, one rank per GPU), --scaling strong (default): the SAME
proteome is split by residues into N protein ranges (configs[2]: "protein-
sharded across 8xMI355X"); one step builds ONE index over all of it
(dbi_build_sharded): each rank digests its range, routes every record to the
rank owning its mass key over RCCL (grouped point-to-point sends over xGMI),
and each owner sorts + de-duplicates its key range.  Every rank holds the whole
proteome in HBM before the timed region (each rank reads the same FASTA: input
staging; the owner merge compares peptide strings of any protein).  After the
timed steps the owners' slices are all-gathered onto every rank
(dbi_shard_replicate, north_star's all-gatherv; timed separately) and every
rank answers its own 1M-query batch locally.  --scaling weak: each rank its own
proteome of the same size (seed + 1000*rank), still one merged index.
--no-merge: independent shard-local indexes instead.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--config swissprot|human|1k|semi|trembl]
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from dbindex_amd.params import DBIndexSearchParams  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BASELINE_METRIC = "peptides indexed/sec + mass-window queries/sec, SwissProt-scale FASTA"
# name -> (description, synthetic proteome (fasta.CONFIGS), params, CPU-baseline sample proteins)
WORKLOADS = {
    "human": ("UniProt-human-scale synthetic proteome (20,000 proteins, seed 2), trypsin, "
              "2 missed cleavages, 500-6000 Da MH+ (BASELINE.json configs[1])", "human",
              lambda: DBIndexSearchParams.trypsin(2), 20000),
    "1k": ("1k-protein synthetic proteome (seed 1), trypsin, 0 missed cleavages (configs[0])", "1k",
           lambda: DBIndexSearchParams.trypsin(0), 1000),
    "swissprot": ("SwissProt-scale synthetic proteome (560,000 proteins, seed 3), trypsin, "
                  "2 missed cleavages (configs[2])", "swissprot",
                  lambda: DBIndexSearchParams.trypsin(2), 100000),
    "semi": ("SwissProt-scale synthetic proteome (560,000 proteins, seed 3), semi-tryptic, "
             "2 missed cleavages + 1M precursor-mass queries +-20 ppm (configs[3])", "swissprot",
             lambda: DBIndexSearchParams.semi_tryptic(2), 5000),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def stdout_to_stderr(fn):
    """Runs fn with fd 1 pointed at stderr (RCCL prints a version banner on
    stdout at init; the bench's stdout carries exactly one JSON line)."""
    import ctypes
    libc = ctypes.CDLL(None)
    sys.stdout.flush()
    libc.fflush(None)
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        return fn()
    finally:
        sys.stdout.flush()
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="swissprot", choices=sorted(WORKLOADS) + ["trembl"])
    ap.add_argument("--trembl-proteins", type=int, default=50_000_000,
                    help="--config trembl: proteins of the whole synthetic proteome (split over the ranks)")
    ap.add_argument("--queries", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold / end-to-end legs")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="engine option (dbi_set_option: tuning switches for experiments), repeatable")
    ap.add_argument("--no-merge", action="store_true",
                    help="N>1: shard-local indexes (no exchange) instead of one merged index")
    ap.add_argument("--merge", action="store_true", help="N=1: run the sharded (RCCL) build with one rank")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="N>1 merged builds: split one proteome over the ranks (strong) or one proteome per rank")
    args = ap.parse_args()

    options = {}
    for o in args.option:
        k, _, v = o.partition("=")
        options[k] = int(v) if v.lstrip("-").isdigit() else v
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    from dbindex_amd import fasta
    from dbindex_amd._native import DeviceBuffer, synchronize
    from dbindex_amd.engine import Engine
    from dbindex_amd.params import DBIndexSearchParams

    coord = None
    merge = (world > 1 and not args.no_merge) or args.merge
    if world > 1:
        # host coordination (barrier, max time, sums, the RCCL id) over plain
        # sockets (dbindex_amd/coord.py): no torch in this process, so the one
        # HIP runtime and the one RCCL mapped are /opt/rocm's, the library's own
        # (checked: _native.check_single_runtime); the data path runs over RCCL
        from dbindex_amd.coord import Coordinator
        coord = Coordinator(world, rank)
    # one GPU per rank; with fewer visible GPUs than local ranks (a rehearsal of
    # the N-rank driver on a small box) ranks share devices -- RCCL refuses
    # that, so only --no-merge runs there
    from dbindex_amd._native import device_count
    ndev = device_count()
    dev = local_rank % ndev if ndev else local_rank
    if args.config == "trembl":
        return run_trembl(args, world, rank, dev, coord, options)

    desc, proteome, make_params, cpu_sample = WORKLOADS[args.config]
    strong = merge and args.scaling == "strong"
    base = dict(fasta.CONFIGS[proteome])
    if not strong:
        base["seed"] = base["seed"] + 1000 * rank  # weak: each rank its own proteome of equal size
    t0 = time.time()
    pp = fasta.synthetic(with_defs=False, **base)
    log(f"[rank {rank}] synthetic {args.config}: P={pp.n_proteins} R={pp.n_residues} ({time.time() - t0:.1f}s)")
    prm = make_params()

    eng = Engine(prm, device=dev, options=options)
    t_ag = 0.0
    if merge:
        from dbindex_amd import shard
        import ctypes
        from dbindex_amd._native import lib as _lib
        uid = stdout_to_stderr(shard.ShardComm.unique_id) if rank == 0 else None
        if world > 1:
            uid = bytes.fromhex(coord.broadcast(uid.hex() if uid else None))
        comm = stdout_to_stderr(lambda: shard.ShardComm(uid, world, rank, dev))
        if strong:
            # every rank holds the whole proteome (the same FASTA); rank r
            # digests its residue-balanced protein range
            R_all, P_all = pp.n_residues, pp.n_proteins
            d_res = DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), dev)
            d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), dev)
            p_begin, p_end = shard.protein_ranges(pp.offsets, world)[rank]
        else:
            # global layout: every rank's residues and offsets, in rank order
            sizes = coord.allgather([pp.n_residues, pp.n_proteins]) if world > 1 else [[pp.n_residues, pp.n_proteins]]
            res_base = np.concatenate([[0], np.cumsum([x[0] for x in sizes])]).astype(np.uint64)
            prot_base = np.concatenate([[0], np.cumsum([x[1] for x in sizes])]).astype(np.int64)
            R_all, P_all = int(res_base[-1]), int(prot_base[-1])
            # every rank's protein offsets, rebased, all-gathered over RCCL
            d_offs = DeviceBuffer(8 * P_all, dev)
            mine_off = DeviceBuffer.from_numpy((pp.offsets[:-1].astype(np.uint64) + res_base[rank]), dev)
            comm.allgatherv(mine_off.ptr, d_offs.ptr, [8 * int(x[1]) for x in sizes])
            off_all = np.concatenate([d_offs.download(np.uint64, P_all), np.array([R_all], np.uint64)])
            del d_offs, mine_off
            # input staging (untimed): every shard's residues into every GPU's HBM
            d_res = DeviceBuffer(R_all + 16, dev)
            mine = d_res.ptr + int(res_base[rank])
            _lib().dbi_dev_copy_h2d(dev, ctypes.c_void_p(mine), pp.residues.ctypes.data_as(ctypes.c_void_p),
                                    pp.n_residues)
            t_ag = time.perf_counter()
            comm.allgatherv(mine, d_res.ptr, [x[0] for x in sizes])
            t_ag = time.perf_counter() - t_ag
            d_off = DeviceBuffer.from_numpy(off_all, dev)
            p_begin, p_end = int(prot_base[rank]), int(prot_base[rank + 1])
        synchronize(dev)
        my_res = int(pp.offsets[p_end] - pp.offsets[p_begin]) if strong else pp.n_residues
        my_prot = p_end - p_begin
        log(f"[rank {rank}] merged index over {P_all} proteins / {R_all} residues; this rank digests proteins "
            f"[{p_begin}, {p_end}) ({my_res} residues)")

        def step():
            return shard.build_sharded(eng, comm, d_res.ptr, R_all, d_off.ptr, P_all, p_begin, p_end)
    else:
        # inputs resident in HBM before the timed region
        d_res = DeviceBuffer.from_numpy(pp.residues, dev)
        d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), dev)
        synchronize(dev)
        my_res, my_prot = pp.n_residues, pp.n_proteins

        def step():
            return eng.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)

    def accumulate(acc):
        for name, ms, by in eng.stage_times():
            a = acc.setdefault(name, [0.0, 0.0, 0])
            a[0] += ms
            a[1] += by
            a[2] += 1

    # warmup: every stage carries HIP events in its dispatch packet -> the
    # per-kernel breakdown and the dominant kernel
    # (the first build is cold: slot count + bounded digest; the second may grow the bounded
    # digest's reservation and run it twice: neither is a steady-state build).
    # The last two warmup builds already time only the dominant kernel, as the
    # timed region does: the engine captures its warm build as a hipGraph on
    # the second identical build and replays it from then on (W >= 4).
    eng.set_timing(True)
    warm_acc = {}
    n_warm = max(args.warmup, 1)
    skip = min(2, n_warm - 1)
    n_dom = 2 if n_warm >= 4 else 0
    dominant = ""
    # the dominant kernel: the longest launch (a stage launched several times
    # per build, such as the three radix scatters, counts per launch)
    def longest(acc):
        return max(acc.items(), key=lambda kv: kv[1][0] / max(kv[1][2], 1))[0] if acc else ""

    for i in range(n_warm):
        if i == n_warm - n_dom:
            dominant = longest(warm_acc)
            eng.set_timing(True, only=dominant)
        st = step()
        if skip <= i < n_warm - n_dom:
            accumulate(warm_acc)
    synchronize(dev)
    if not n_dom:
        dominant = longest(warm_acc)

    # timed region: events only on the dominant kernel (each timed stage costs
    # a few us of dispatch overhead; the other stages run untimed)
    eng.set_timing(True, only=dominant)
    stage_acc = {}
    if world > 1:
        coord.barrier()
    synchronize(dev)
    if merge:
        t_start = time.perf_counter()
        n_total = 0
        shard_acc = []
        for _ in range(args.steps):
            st = step()
            n_total += st.n_total
            accumulate(stage_acc)
            shard_acc.append((st.digest_ms, st.partition_ms, st.exchange_ms, st.merge_ms))
    else:
        # single-device builds: the C entry point with its arguments bound once
        # and the dominant stage's event time read into preallocated arrays --
        # the Python bookkeeping per build (stats and stage tables as objects,
        # ~45 us between builds in the kernel trace) is left out of the loop.
        # The builds are identical: their stats are read once after it.
        import ctypes
        from dbindex_amd import _native
        lib = _native.lib()
        c_args = (eng.h, ctypes.c_void_p(d_res.ptr), ctypes.c_uint64(pp.n_residues), ctypes.c_void_p(d_off.ptr),
                  ctypes.c_uint64(pp.n_proteins), None)
        names = [n for n, _, _ in eng.stage_times()]
        k = len(names)
        ms_buf, by_buf = np.zeros(max(k, 1)), np.zeros(max(k, 1))
        ms_p, by_p = ms_buf.ctypes.data_as(ctypes.c_void_p), by_buf.ctypes.data_as(ctypes.c_void_p)
        n_st = ctypes.c_uint64()
        dom_i = names.index(dominant) if dominant in names else -1
        dom_ms = dom_by = 0.0
        t_start = time.perf_counter()
        for _ in range(args.steps):
            rc = lib.dbi_build_device(*c_args)
            if rc:
                _native.check(rc)
            if dom_i >= 0:
                lib.dbi_stage_times(eng.h, None, ms_p, by_p, ctypes.c_uint64(k), ctypes.byref(n_st))
                dom_ms += ms_buf[dom_i]
                dom_by += by_buf[dom_i]
        synchronize(dev)
        st = eng.stats()
        n_total = st.n_total * args.steps
        if [n for n, _, _ in eng.stage_times()] != names:
            raise RuntimeError("the timed builds ran another stage table than the warmup's last build")
        if dom_i >= 0:
            stage_acc[dominant] = [dom_ms, dom_by, args.steps]
    synchronize(dev)
    if world > 1:
        coord.barrier()
    elapsed = time.perf_counter() - t_start

    # whole-job: units of all ranks (each rank's digested occurrences; a
    # strong-scaling step counts the proteome once) / max time over ranks
    if world > 1:
        elapsed = coord.allreduce([elapsed], "max")[0]
        n_total_all = coord.allreduce([n_total], "sum")[0]
    else:
        n_total_all = float(n_total)
    value = n_total_all / elapsed if elapsed > 0 else 0.0
    ms_per_step = 1000.0 * elapsed / max(args.steps, 1)

    def kernel_table(acc, builds):
        out = []
        for name, (ms, by, cnt) in acc.items():
            if ms <= 0:
                continue
            # several launches per build share a name (radix passes): per-launch averages
            out.append(dict(kernel=name, launches=cnt, ms_per_build=ms / builds, avg_ms=ms / cnt,
                            alg_bytes=by / cnt, gbps=(by / cnt) / (ms / cnt * 1e-3) / 1e9))
        out.sort(key=lambda k: -k["ms_per_build"])
        return out

    def pmc_summary():
        """The newest committed rocprofv3 PMC summary of this workload
        (profiles/<round>_<config>_summary.json, tools/prof_summary.py:
        2 x FETCH_SIZE + WRITE_SIZE per launch, degenerate launches left out,
        and the build's summed traffic), or (None, None)."""
        files = round_profiles(f"*_{args.config}_summary.json")
        for f in reversed(files):
            d = json.load(open(f))
            if d.get("stages"):
                return d, os.path.relpath(f, ROOT)
        return None, None

    kernels = kernel_table(warm_acc, max(n_warm - skip - n_dom, 1))
    timed = kernel_table(stage_acc, args.steps)
    dom = timed[0] if timed else None
    build_alg = my_res + 8.0 * (my_prot + 1) + 48.0 * st.n_total  # SURVEY.md §8(d), this rank's share
    est = eng.stats()  # merged: this rank's owner slice
    if merge:
        unique_all, keys_all = st.g_unique, st.g_keys
        ph = np.mean(np.array(shard_acc), axis=0) if shard_acc else np.zeros(4)
        phases = dict(zip(("digest_ms", "partition_ms", "exchange_ms", "merge_ms"), map(float, ph)))
        if not strong:
            phases["residue_allgather_ms_untimed"] = t_ag * 1e3
        phases["owner_records"] = st.n_received
        phases["records_sent"] = st.n_sent
    else:
        unique_all, keys_all, phases = st.n_unique, st.n_keys, None

    # secondary: mass-window queries/sec on the built index (1M queries, +-20 ppm)
    qps = None
    if args.queries > 0 and merge:
        # north_star's all-gatherv: every owner's slice onto every rank, then
        # every rank answers its own 1M batch locally (no exchange per batch)
        if world > 1:
            coord.barrier()
        synchronize(dev)
        t_rep = time.perf_counter()
        shard.replicate(eng, comm)
        synchronize(dev)
        t_rep = time.perf_counter() - t_rep
        if world > 1:
            t_rep = coord.allreduce([t_rep], "max")[0]
        rst = eng.stats()
        ex = eng.export()["mass"]
        rng = np.random.Generator(np.random.PCG64(7 + rank))
        nq = args.queries
        k = int(nq * 0.9)
        m = np.empty(nq)
        m[:k] = ex[rng.integers(0, ex.shape[0], k)] * (1 + rng.normal(0, 5e-6, k)) if ex.shape[0] else 1000.0
        m[k:] = rng.uniform(500, 6000, nq - k)
        tol = m * (1 - 1 / (20.0 / 1e6 + 1))
        dm, dt = DeviceBuffer.from_numpy(m, dev), DeviceBuffer.from_numpy(tol, dev)
        df, dc = DeviceBuffer(8 * nq, dev), DeviceBuffer(8 * nq, dev)
        synchronize(dev)
        eng.query_prepare()
        for _ in range(3):
            eng.query_device(dm.ptr, dt.ptr, nq, df.ptr, dc.ptr)
        synchronize(dev)
        reps = 20
        if world > 1:
            coord.barrier()
        tq = time.perf_counter()
        for _ in range(reps):
            eng.query_device(dm.ptr, dt.ptr, nq, df.ptr, dc.ptr)
        synchronize(dev)
        if world > 1:
            coord.barrier()
        tq = time.perf_counter() - tq
        hits = int(dc.download(np.uint64, nq).sum())
        if world > 1:
            tq = coord.allreduce([tq], "max")[0]
        qps = dict(value=world * nq * reps / tq, unit="queries/s", queries_per_rank=nq, tol_ppm=20.0,
                   avg_hits=hits / nq, kind="range lookup on each rank's replica of the whole index",
                   index=f"the merged index above, replicated onto all {world} ranks "
                         f"(dbi_shard_replicate: {rst.n_unique} unique peptides, {rst.n_kept} occurrences)",
                   replicate_ms=1e3 * t_rep,
                   replicate_bytes_per_rank=int(20 * rst.n_unique + 4 * rst.n_kept))
    if args.queries > 0 and not merge:
        ex = eng.export()["mass"]
        rng = np.random.Generator(np.random.PCG64(7 + rank))
        nq = args.queries
        k = int(nq * 0.9)
        m = np.empty(nq)
        m[:k] = ex[rng.integers(0, ex.shape[0], k)] * (1 + rng.normal(0, 5e-6, k))
        m[k:] = rng.uniform(500, 6000, nq - k)
        tol = m * (1 - 1 / (20.0 / 1e6 + 1))
        dm, dt = DeviceBuffer.from_numpy(m, dev), DeviceBuffer.from_numpy(tol, dev)
        df, dc = DeviceBuffer(8 * nq, dev), DeviceBuffer(8 * nq, dev)
        synchronize(dev)
        t_q = time.perf_counter()
        eng.query_prepare()  # directory of the index of the last timed build
        qdir_ms = 1e3 * (time.perf_counter() - t_q)
        for _ in range(3):
            eng.query_device(dm.ptr, dt.ptr, nq, df.ptr, dc.ptr)
        synchronize(dev)
        reps = 20
        tq = time.perf_counter()
        for _ in range(reps):
            eng.query_device(dm.ptr, dt.ptr, nq, df.ptr, dc.ptr)
        synchronize(dev)
        tq = time.perf_counter() - tq
        hits = int(dc.download(np.uint64, nq).sum())
        qps = dict(value=nq * reps / tq, unit="queries/s", queries=nq, tol_ppm=20.0, avg_hits=hits / nq,
                   kind="range lookup: (first, count) of every window's run of unique ids (the complete "
                        "answer over the mass-sorted unique table), device in/out",
                   index="the build above", qdir_build_ms=qdir_ms)
        # hit-producing leg: every hit's unique id and protein ids materialised in
        # HBM, all nq windows, in consecutive batches of at most ~40 GB of hit
        # buffers (semi-tryptic windows hold ~20x more hits than tryptic ones)
        counts = dc.download(np.uint64, nq).astype(np.float64)
        qps["materialised"] = hits_leg(eng, dm, dt, nq, counts)

    cold = None
    if rank == 0 and world == 1 and not merge and not args.no_cold:
        # the reference's real use is a one-off build (DBIndexer.run): the cold
        # pipeline (no capacities, grids, map or graph from earlier builds),
        # and FASTA file -> index end to end
        cold = cold_legs(eng, prm, pp, d_res, d_off, dev, args.config, options)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # reference-semantics CPU restatement (oracle/cpu_ref.cpp) on a bounded
        # sample of the same workload: one thread per host core (protein ranges,
        # then row ranges) and single-threaded like the reference
        sample = pp.slice(0, min(cpu_sample, pp.n_proteins))
        cpu = cpu_baseline_legs(prm, sample)
        oix = cpu.pop("_oix")
        cpu["queries"] = cpu_query_legs(oix, args.queries or 1_000_000)
        cpu["sample_parity"] = sample_parity(prm, sample, oix, dev, options)

    from dbindex_amd._native import runtime_info
    runtime = runtime_info()  # raises if two HIP runtimes / RCCLs are mapped
    prof, prof_src = pmc_summary()
    dom_prof = (prof or {}).get("stages", {}).get(dom["kernel"], {}) if dom else {}
    build_traffic = ((prof or {}).get("build") or {}).get("traffic_bytes") if not merge else None
    copy_gbps = hbm_copy_gbps(dev) if rank == 0 else None
    build_gbps = build_alg / (ms_per_step * 1e-3) / 1e9
    if rank == 0:
        out = {
            "metric": BASELINE_METRIC,
            "value": value,
            "unit": "peptides indexed/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            # N>1 default: one proteome split over the ranks (total work fixed);
            # --no-merge / --scaling weak: one proteome per rank
            "scaling": "weak" if (args.no_merge or args.scaling == "weak") else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded proteome, SwissProt residue frequencies; SURVEY.md §8(d))",
            "config": {
                "workload": desc + (
                    ", single GPU" if world == 1 and not merge else
                    f", {'one proteome split by residues over' if strong else 'one proteome per rank on'} {world} "
                    f"GPU{'s' if world > 1 else ''}, " + ("one merged index (RCCL owner exchange)" if merge
                                                          else "shard-local indexes")),
                "proteins_per_gpu": my_prot,
                "residues_per_gpu": my_res,
                "proteins": pp.n_proteins * (world if merge and not strong else 1),
                "peptides_per_step_per_gpu": st.n_total,
                "unique_peptides": unique_all,
                "mass_keys": keys_all,
                "parallelism": (f"protein-sharded x{world} ({'one proteome split' if strong else 'one proteome per rank'}), "
                                f"one index: RCCL owner exchange by mass key" if merge
                                else f"protein-sharded x{world}, shard-local indexes" if world > 1 else "single GPU"),
                "n_bins": est.n_bins,
                "n_big_bins": est.n_big_bins,
            },
            # the headline fraction is the WHOLE BUILD's: SURVEY.md §8(d)'s
            # algorithmic bytes over the timed ms per build; the longest kernel
            # (HIP events in its dispatch packets inside the timed region) beside it
            "roofline": {
                "bound": "hbm",
                "scope": "whole build (this rank's share at N>1)",
                "achieved": build_gbps,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": build_gbps / HBM_PEAK_GBPS,
                "traffic": build_traffic,
                "traffic_source": prof_src if build_traffic else None,
                "traffic_note": "PMC HBM bytes per build: every build stage's 2 x FETCH_SIZE + WRITE_SIZE per "
                                "launch x launches per build (tools/prof_summary.py, degenerate launches dropped)",
                "alg_bytes": build_alg,
                "formula": "R + 8(P+1) + 48N (SURVEY.md §8(d))",
                "measured_copy_gbps": copy_gbps,  # STREAM-like copy on this GPU: the reachable ceiling
                "frac_of_measured_copy": build_gbps / copy_gbps if copy_gbps else None,
                "kernel": None if dom is None else {
                    "name": dom["kernel"],
                    "achieved": dom["gbps"],
                    "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s",
                    "frac": dom["gbps"] / HBM_PEAK_GBPS,
                    "traffic": dom_prof.get("traffic_bytes"),
                    "traffic_source": prof_src if "traffic_bytes" in dom_prof else None,
                    "alg_bytes_per_launch": dom["alg_bytes"],
                    "avg_launch_ms": dom["avg_ms"],
                    "rocprof_avg_launch_ms": dom_prof["avg_us"] / 1e3 if "avg_us" in dom_prof else None,
                    "frac_of_measured_copy": dom["gbps"] / copy_gbps if copy_gbps else None,
                },
            },
            # the chunk sort runs as three kernels (chunk_sort, chunk_sort_mid for
            # chunks with a bin above the one-wave sort, chunk_sort_big above
            # CHUNK_CAP); together: 16 B in + 16 B out per record per build
            "chunk_sort_family": chunk_family(kernels, st.n_total),
            "kernels": kernels,
            "kernels_note": "per-kernel HIP events (dispatch-packet start/stop) over the warmup builds; "
                            "roofline.kernel (the longest launch) is re-timed inside the timed region",
            "sharded_phases": phases,
            "queries": qps,
            # the one-off build: cold pipeline, first build with allocations, FASTA file -> index
            "cold": cold,
            "cpu_baseline": cpu,
            # the HIP runtime and RCCL this process runs on (one of each: checked)
            "runtime": runtime,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if coord is not None:
        coord.close()


def chunk_family(kernels, n_total):
    """The chunk-sort stages combined (warmup events, per build): time, 32 B per
    record, fraction of the HBM peak."""
    ms = sum(k["ms_per_build"] for k in kernels if k["kernel"].startswith("chunk_sort"))
    if ms <= 0:
        return None
    alg = 32.0 * n_total
    return dict(stages=[k["kernel"] for k in kernels if k["kernel"].startswith("chunk_sort")],
                ms_per_build=ms, alg_bytes=alg, achieved=alg / (ms * 1e-3) / 1e9, peak=HBM_PEAK_GBPS,
                unit="GB/s", frac=alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS)


def host_threads() -> int:
    """Host threads for the all-cores CPU leg: the cores this process may use
    (OMP_NUM_THREADS caps it: the GPU box's CPU share), one per core."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else max(1, n)


def cpu_baseline_legs(prm, sample) -> dict:
    from oracle import cref
    nthreads = host_threads()
    cp = prm.to_c()
    with cref.threads(nthreads):
        t_all = time.perf_counter()
        oix = cref.Index(cp, sample.residues, sample.offsets)
        t_all = time.perf_counter() - t_all
    t_one = time.perf_counter()
    one = cref.Index(cp, sample.residues, sample.offsets)
    t_one = time.perf_counter() - t_one
    assert one.n_total == oix.n_total and one.n_unique == oix.n_unique
    del one
    desc = (f"{sample.n_proteins} proteins / {sample.n_residues} residues of the same workload "
            f"({oix.n_total} peptides)")
    return dict(value=oix.n_total / t_all, unit="peptides indexed/s", cores=nthreads, kind="port",
                sample=f"{desc}: oracle/cpu_ref.cpp restatement, digest over protein ranges + merge over row "
                       f"ranges, {nthreads} threads, {t_all:.2f}s",
                seconds=t_all, nproc=os.cpu_count(), host_cpu=cpu_model(),
                single_core=dict(value=oix.n_total / t_one, unit="peptides indexed/s", cores=1, kind="port",
                                 seconds=t_one, sample=f"{desc}, one thread (the reference's threading)"),
                _oix=oix)


def cold_legs(eng, prm, pp, d_res, d_off, dev: int, config: str, options=None) -> dict:
    """The one-off build (DBIndexer.java:508-684) beside the warm steady state:
    cold_ms -- this engine forced cold (dbi_set_cold: slot count + bounded digest,
    radix tail, full list grids; buffers kept), best of 3; first_build_ms -- a
    fresh engine's first build (its allocations included); end_to_end -- a
    FASTA file of the proteome written to a temporary directory (untimed),
    then dbi_fasta_read (multi-threaded parser) + a fresh engine's dbi_build
    (H2D of residues and offsets + the cold build), SURVEY.md §8(d)."""
    import tempfile
    from dbindex_amd import fasta
    from dbindex_amd._native import synchronize
    from dbindex_amd.engine import Engine

    def build_dev(e):
        return e.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)

    eng.set_timing(False)
    ts = []
    for _ in range(3):
        eng.set_cold()
        synchronize(dev)
        t = time.perf_counter()
        st = build_dev(eng)
        synchronize(dev)
        ts.append(1e3 * (time.perf_counter() - t))
    out = dict(cold_ms=min(ts), cold_ms_runs=ts, peptides=st.n_total,
               cold_peptides_per_s=st.n_total / (min(ts) * 1e-3),
               cold_kind="dbi_set_cold on the benched engine: slot count + bounded digest, radix tail, full list grids "
                         "(device buffers kept)")
    if st.n_total > 200_000_000:  # (semi-tryptic: a second engine's ~100 GB would not fit beside this one)
        out["first_build_ms"] = out["end_to_end"] = None
        out["note"] = "fresh-engine legs skipped: a second index of this size does not fit beside the benched one"
        return out
    with Engine(prm, device=dev, options=options) as e2:
        e2.set_timing(False)
        synchronize(dev)
        t = time.perf_counter()
        build_dev(e2)
        synchronize(dev)
        out["first_build_ms"] = 1e3 * (time.perf_counter() - t)
    # end to end: FASTA text -> packed proteome -> index
    threads = host_threads()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, f"{config}.fasta")
        t = time.perf_counter()
        with open(path, "w") as fh:
            fasta.write_fasta(pp, fh)
        write_s = time.perf_counter() - t
        size = os.path.getsize(path)
        t0 = time.perf_counter()
        rp = fasta.read_fasta(path, threads=threads, with_defs=False)
        t1 = time.perf_counter()
        with Engine(prm, device=dev, options=options) as e3:
            e3.set_timing(False)
            t_open = time.perf_counter()
            st3 = e3.build(rp)
            synchronize(dev)
            t_built = time.perf_counter()
        t2 = time.perf_counter()
    same = rp.n_proteins == pp.n_proteins and rp.n_residues == pp.n_residues and st3.n_total == st.n_total
    # end to end = FASTA file -> index resident in HBM, ready for queries
    # (DBIndexer.run then keeps it); the engine's teardown is reported apart
    out["end_to_end"] = dict(ms=1e3 * (t_built - t0), fasta_read_ms=1e3 * (t1 - t0), build_ms=1e3 * (t_built - t1),
                             open_ms=1e3 * (t_open - t1), dbi_build_ms=1e3 * (t_built - t_open),
                             close_ms_not_included=1e3 * (t2 - t_built),
                             fasta_bytes=size, fasta_write_s_untimed=write_s, parser_threads=threads,
                             peptides_per_s=st3.n_total / (t_built - t0), same_proteome=bool(same),
                             kind="dbi_fasta_read of the written FASTA, then a fresh engine's dbi_build "
                                  "(host residues: H2D + cold build, allocations included)")
    return out


def cpu_query_legs(oix, nq: int) -> dict:
    """getSequences(m, tol) windows (DBIndexer.java:762-844 ->
    IndexMerge.getSequences :146-217, as oracle/cpu_ref.cpp restates them) over
    the CPU sample's index: the same +-20 ppm query mix, all cores and one."""
    from oracle import cref
    rng = np.random.Generator(np.random.PCG64(7))
    ex = oix.unique()["mass"]
    k = int(nq * 0.9)
    m = np.empty(nq)
    m[:k] = ex[rng.integers(0, ex.shape[0], k)] * (1 + rng.normal(0, 5e-6, k))
    m[k:] = rng.uniform(500, 6000, nq - k)
    tol = m * (1 - 1 / (20.0 / 1e6 + 1))
    nthreads = host_threads()
    with cref.threads(nthreads):
        t = time.perf_counter()
        _, cnt = oix.query_batch(m, tol)
        t_all = time.perf_counter() - t
    n1 = min(nq, 200_000)  # one thread: a bounded share of the same windows
    t = time.perf_counter()
    oix.query_batch(m[:n1], tol[:n1])
    t_one = time.perf_counter() - t
    return dict(value=nq / t_all, unit="queries/s", cores=nthreads, kind="port", queries=nq,
                avg_hits=float(cnt.mean()), seconds=t_all,
                sample=f"{nq} +-20 ppm windows over the sample's index ({oix.n_unique} unique peptides): "
                       "oracle/cpu_ref.cpp getSequences restatement, (first, count) per window",
                single_core=dict(value=n1 / t_one, unit="queries/s", cores=1, queries=n1, seconds=t_one))


def sample_parity(prm, sample, oix, dev: int, options=None) -> dict:
    """The CPU leg's sample built on the GPU too: counts and a digest of every
    index array equal the oracle's (bit-exact)."""
    import hashlib
    from dbindex_amd.engine import Engine

    def digest(d):
        h = hashlib.sha256()
        for k in ("mass", "prot_id", "offset", "length", "occ_off", "occ_prot"):
            a = np.ascontiguousarray(d[k])
            h.update(a.view(np.uint64).tobytes() if k == "mass" else a.astype(np.uint64).tobytes())
        return h.hexdigest()[:16]

    with Engine(prm, device=dev, options=options) as e2:
        st = e2.build(sample)
        g = digest(e2.export())
    o = digest(oix.unique())
    same = (st.n_total == oix.n_total and st.n_unique == oix.n_unique and st.n_keys == oix.n_keys and g == o)
    return dict(ok=bool(same), gpu_sha=g, oracle_sha=o, n_total=st.n_total, n_unique=st.n_unique)


def hit_batches(counts, cap_bytes: float = 40e9, per_hit: float = 12.0):
    """Consecutive query ranges [a, b) whose hits (range-lookup counts) take at
    most cap_bytes of hit buffers each (a single window above it: alone)."""
    cum = np.concatenate([[0.0], np.cumsum(counts * per_hit)])
    out, a, n = [], 0, len(counts)
    while a < n:
        b = int(np.searchsorted(cum, cum[a] + cap_bytes, side="right")) - 1
        b = min(max(b, a + 1), n)
        out.append((a, b))
        a = b
    return out


def hits_leg(eng, dm, dt, nq: int, counts, reps: int = 3) -> dict:
    """nq +-20 ppm windows through dbi_query_hits_device: per query its unique
    ids, per hit its protein ids (occurrence CSR), all written to HBM, batch
    by batch (hit_batches) when the hits of all windows exceed the buffer cap.
    Algorithmic bytes: 32 Q (mass + tol in, two u64 offsets
    out) + 12 H (id out, protein-list start out, occ_off read) + 8 Ho (protein
    id read + written), Ho = protein ids of all hits; also SURVEY.md §8(d)'s
    16 Q + 16 H."""
    from dbindex_amd._native import synchronize
    batches = hit_batches(counts)
    for a, b in batches[:1]:  # warm: grows the buffers
        eng.query_hits_device(dm.ptr + 8 * a, dt.ptr + 8 * a, b - a)
    synchronize(eng.device)
    H = Ho = 0
    t = 0.0
    for a, b in batches:
        eng.query_hits_device(dm.ptr + 8 * a, dt.ptr + 8 * a, b - a)  # this batch's buffer sizes
        synchronize(eng.device)
        t0 = time.perf_counter()
        for _ in range(reps):
            r = eng.query_hits_device(dm.ptr + 8 * a, dt.ptr + 8 * a, b - a)
        synchronize(eng.device)
        t += (time.perf_counter() - t0) / reps
        H += r.n_hits
        Ho += r.n_prot_ids
    alg = 32.0 * nq + 12.0 * H + 8.0 * Ho
    alg_s = 16.0 * nq + 16.0 * H
    return dict(value=nq / t, unit="queries/s", ms_per_batch=1e3 * t, queries=nq, hits=H, protein_ids=Ho,
                batches=len(batches),
                kind="materialised: unique ids + protein ids of every hit in HBM (dbi_query_hits_device), all "
                     "windows, in batches of at most ~40 GB of hit buffers",
                roofline=dict(bound="hbm", alg_bytes=alg, formula="32Q + 12H + 8Ho",
                              achieved=alg / t / 1e9, peak=HBM_PEAK_GBPS, unit="GB/s",
                              frac=alg / t / 1e9 / HBM_PEAK_GBPS,
                              survey_formula="16Q + 16H (SURVEY.md §8(d))", survey_alg_bytes=alg_s,
                              survey_frac=alg_s / t / 1e9 / HBM_PEAK_GBPS))


def hbm_copy_gbps(dev: int, nbytes: int = 1 << 31, reps: int = 10):
    """Measured device-copy bandwidth (read + write bytes / s, dbi_hbm_copy_bandwidth), GB/s."""
    import ctypes
    from dbindex_amd._native import lib as _lib
    v = ctypes.c_double(0.0)
    rc = _lib().dbi_hbm_copy_bandwidth(dev, nbytes, reps, ctypes.byref(v))
    return v.value if rc == 0 else None


def run_trembl(args, world: int, rank: int, dev: int, coord, options=None) -> None:
    """BASELINE.json configs[4]: TrEMBL-scale synthetic proteome (50M proteins,
    ~1.8e10 residues), non-specific digestion 6-50, COUNT only: ~7e11 peptide
    occurrences (~12 TB of records) cannot be materialised, so a step digests
    this rank's proteins in COUNT mode (dbi_count: totalSeqCount).  The whole
    proteome is split over the ranks (strong scaling); each rank generates its
    range on its own GPU (dbi_synth_proteome, counter-based: no data moves)
    into HBM before the timed region, in chunks of < 2^32 residues."""
    import ctypes

    from dbindex_amd import fasta
    from dbindex_amd._native import DeviceBuffer, synchronize
    from dbindex_amd.engine import Engine

    seed, P = 4, int(args.trembl_proteins)
    p0, p1 = P * rank // world, P * (rank + 1) // world
    tables = fasta.synth_tables()
    prm = DBIndexSearchParams.non_specific(50)
    eng = Engine(prm, device=dev, options=options)
    nb = int(prm.index_factor)  # SQLiteMult buckets (+1: past the last one)
    comm = None
    if world > 1:  # the per-bucket counts are summed over the ranks by RCCL (ncclAllReduce)
        from dbindex_amd import shard
        uid = stdout_to_stderr(shard.ShardComm.unique_id) if rank == 0 else None
        uid = bytes.fromhex(coord.broadcast(uid.hex() if uid else None))
        comm = stdout_to_stderr(lambda: shard.ShardComm(uid, world, rank, dev))
    zeros = np.zeros(nb + 1, np.uint64)
    d_hist = DeviceBuffer.from_numpy(zeros, dev)      # this rank's buckets, per step
    d_hist_all = DeviceBuffer.from_numpy(zeros, dev)  # every rank's (allreduce)
    t0 = time.time()
    base = fasta.synth_residue_base(seed, p0, tables[0])
    CH = 1 << 20  # proteins per chunk (~3.8e8 residues)
    chunks = []
    n_res_all = 0
    lens_total = 0
    for a in range(p0, p1, CH):
        lens_total += int(fasta.synth_lengths(seed, a, min(CH, p1 - a), tables[0]).sum())
    d_res_all = DeviceBuffer(lens_total + 16, dev)
    d_off_all = DeviceBuffer(8 * ((p1 - p0) + (p1 - p0 + CH - 1) // CH + 1), dev)
    off_pos = 0
    for a in range(p0, p1, CH):
        n = min(CH, p1 - a)
        d_res, d_off, n_res = eng.synth_proteome(seed, a, n, base + n_res_all, tables)
        d_res_all.copy_from_device(n_res_all, d_res, n_res)
        d_off_all.copy_from_device(8 * off_pos, d_off, 8 * (n + 1))
        chunks.append((d_res_all.ptr + n_res_all, n_res, d_off_all.ptr + 8 * off_pos, n))
        n_res_all += n_res
        off_pos += n + 1
    synchronize(dev)
    log(f"[rank {rank}] trembl proteins [{p0}, {p1}): {n_res_all} residues in {len(chunks)} chunks, "
        f"generated in HBM ({time.time() - t0:.1f}s)")

    def count_only():
        tot = 0
        for c in chunks:
            tot += eng.count_device(*c)[0]
        return tot

    def step():
        # the configs[4] step: every occurrence counted into
        # its SQLiteMult bucket ((int)m / BUCKET_MASS_RANGE,
        # DBIndexStoreSQLiteMult.java:215-217), the per-bucket counts of all
        # ranks summed by RCCL (ncclAllReduce); totalSeqCount = their sum
        d_hist.upload(zeros)
        tot = 0
        for c in chunks:
            tot += eng.count_buckets_device(*c, d_hist.ptr)[0]
        if comm is not None:
            comm.allreduce_u64(d_hist.ptr, d_hist_all.ptr, nb + 1)
        return tot

    for _ in range(max(args.warmup, 1)):
        n_step = step()
    if world > 1:
        coord.barrier()
    synchronize(dev)
    t = time.perf_counter()
    for _ in range(args.steps):
        n_step = step()
    synchronize(dev)
    if world > 1:
        coord.barrier()
    elapsed = time.perf_counter() - t
    n_all = float(n_step * args.steps)
    if world > 1:
        elapsed = coord.allreduce([elapsed], "max")[0]
        n_all, res_all = coord.allreduce([n_all, float(n_res_all)], "sum")
    else:
        res_all = float(n_res_all)
    hist = (d_hist_all if comm is not None else d_hist).download(np.uint64, nb + 1)
    if int(hist.sum()) * args.steps != int(n_all):
        raise RuntimeError(f"bucket counts {int(hist.sum())} do not add up to totalSeqCount {int(n_all) // args.steps}")
    # beside it: the plain count (totalSeqCount only, dbi_count), timed on its own
    if world > 1:
        coord.barrier()
    synchronize(dev)
    t_c = time.perf_counter()
    n_c = count_only()
    synchronize(dev)
    if world > 1:
        coord.barrier()
    t_c = time.perf_counter() - t_c
    if world > 1:
        t_c = coord.allreduce([t_c], "max")[0]
        n_c = coord.allreduce([float(n_c)], "sum")[0]
    if int(n_c) != int(n_all) // args.steps:
        raise RuntimeError(f"dbi_count {int(n_c)} != the bucket pass's totalSeqCount {int(n_all) // args.steps}")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import cref
        sample = fasta.synth_proteome(seed, 0, 120000, 0, tables)  # ~10 s of single-core count
        cp = prm.to_c()
        nthreads = host_threads()
        with cref.threads(nthreads):
            t_all = time.perf_counter()
            want = cref.count(cp, sample.residues, sample.offsets)[0]
            t_all = time.perf_counter() - t_all
        t1 = time.perf_counter()
        want1 = cref.count(cp, sample.residues, sample.offsets)[0]
        t1 = time.perf_counter() - t1
        assert want1 == want
        desc = (f"cutSeq count (oracle/cpu_ref.cpp) of {sample.n_proteins} proteins / {sample.n_residues} residues "
                f"of the same proteome ({want} peptides)")
        cpu = dict(value=want / t_all, unit="peptides indexed/s", cores=nthreads, kind="port",
                   sample=f"{desc}, {nthreads} threads over protein ranges, {t_all:.2f}s", seconds=t_all,
                   nproc=os.cpu_count(), host_cpu=cpu_model(),
                   single_core=dict(value=want / t1, unit="peptides indexed/s", cores=1, kind="port", seconds=t1,
                                    sample=f"{desc}, one thread"))
        # the same sample counted on the GPU: totalSeqCount parity at this scale
        d_sr = DeviceBuffer.from_numpy(np.concatenate([sample.residues, np.zeros(16, np.uint8)]), dev)
        d_so = DeviceBuffer.from_numpy(sample.offsets.astype(np.uint64), dev)
        g = eng.count_device(d_sr.ptr, sample.n_residues, d_so.ptr, sample.n_proteins)[0]
        cpu.update(gpu_count_same_sample=g, sample_parity=bool(g == want))
        # and its per-bucket counts
        with cref.threads(nthreads):
            want_h = cref.count_buckets(cp, sample.residues, sample.offsets)
        d_h = DeviceBuffer.from_numpy(zeros, dev)
        eng.count_buckets_device(d_sr.ptr, sample.n_residues, d_so.ptr, sample.n_proteins, d_h.ptr)
        cpu["sample_bucket_parity"] = bool(np.array_equal(d_h.download(np.uint64, nb + 1), want_h))
    if rank == 0:
        ms = 1000.0 * elapsed / max(args.steps, 1)
        alg = res_all + 8.0 * (P + 1)  # residues + offsets read once per step (count mode writes nothing)
        print(json.dumps({
            "metric": "peptides indexed/sec (count-only), TrEMBL-scale synthetic FASTA",
            "value": n_all / elapsed, "unit": "peptides indexed/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (counter-based proteome generated on the device, SwissProt residue frequencies)",
            "config": {"workload": f"TrEMBL-scale synthetic proteome ({P} proteins, seed {seed}), non-specific "
                                   f"6-50, count only (BASELINE.json configs[4])",
                       "proteins": P, "residues": res_all, "peptides_per_step": n_all / max(args.steps, 1),
                       "parallelism": (f"protein ranges x{world}, per-bucket counts summed by RCCL allreduce"
                                       if world > 1 else "single GPU")},
            # occurrences per SQLiteMult bucket, (int)m / BUCKET_MASS_RANGE (the last: past the last bucket)
            "bucket_counts": {"bucket_mass_range_da": 8000 // nb, "counts": [int(x) for x in hist],
                              "combined": "ncclAllReduce (dbi_comm_allreduce_u64)" if world > 1 else "one rank",
                              "kind": "the timed step: dbi_count_buckets over every chunk + the allreduce; the "
                                      "last entry is past the last bucket"},
            "count_only": {"ms": 1e3 * t_c, "peptides_per_s": n_c / t_c,
                           "kind": "dbi_count (totalSeqCount only, no buckets) over every chunk, one pass after "
                                   "the timed steps"},
            "roofline": {"bound": "hbm", "kernel": "digest_count",
                         "achieved": alg / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, "traffic": None,
                         "note": "algorithmic HBM bytes per step are R + 8P (no records written): "
                                 f"{alg / 1e9:.1f} GB; the count walk is VALU-bound (~7.5e11 peptide "
                                 "steps per step), so the HBM fraction is tiny by construction"},
            "issue_roofline": trembl_issue_roofline(len(chunks), ms),
            "cpu_baseline": cpu,
        }), flush=True)
    eng.close()
    if comm is not None:
        comm.close()


VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions/s: 256 CUs x 4 SIMDs, one per 2 cycles at 2.4 GHz


def trembl_issue_roofline(chunks_per_step: int, ms: float):
    """configs[4] is VALU-bound, so its roofline is the VALU issue rate
    (VERDICT r04): the bucket-count kernel's SQ_INSTS_VALU per launch from the
    newest profiles/*_trembl_sq.json (tools/sq_kernel_totals.py over a
    rocprofv3 --pmc pass of this bench, tools/gpu_round.sh pmc_sq_trembl) x the
    launches of one step (one per chunk), over the step time, against the
    chip's VALU issue peak (MI355X_MICROARCH.md: a SIMD issues a wave64 VALU
    instruction every 2 cycles)."""
    files = round_profiles("*_trembl_sq.json")
    if not files:
        return None
    d = json.load(open(files[-1]))
    # (the bucket kernel: k_digest_count_cuts<true, true> up to round 5, <true, true, KT> since -- one per
    # tracked-boundary count)
    k = next((v for n, v in d["kernels"].items() if "k_digest_count_cuts<true, true" in n), None)
    if not k or not k.get("launches"):
        return None
    per_launch = k["SQ_INSTS_VALU"] / k["launches"]
    achieved = per_launch * chunks_per_step / (ms * 1e-3)
    return {"bound": "valu", "kernel": "digest_count (bucket pass)", "achieved": achieved, "peak": VALU_ISSUE_PEAK,
            "unit": "wave64 VALU instructions/s", "frac": achieved / VALU_ISSUE_PEAK,
            "valu_per_step": per_launch * chunks_per_step, "source": os.path.relpath(files[-1], ROOT),
            "counts_from": "a separate rocprofv3 --pmc run of this bench (the instruction counts), timed by this run",
            "salu_per_step": k.get("SQ_INSTS_SALU", 0.0) / k["launches"] * chunks_per_step,
            "lds_per_step": k.get("SQ_INSTS_LDS", 0.0) / k["launches"] * chunks_per_step}


def round_profiles(pattern: str):
    """Committed profiles/<tag>_... files matching pattern, oldest first by
    their round tag (r05z < r06a: the file name, not the mtime, which a fresh
    checkout sets in checkout order -- ADVICE r05)."""
    import glob
    return sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=os.path.basename)


if __name__ == "__main__":
    main()
