#!/usr/bin/env python3
"""bench.py — peptides indexed/sec on the MI355X engine (BASELINE.json metric).

Step = one full index build (digest -> mass bins -> per-bin sort + dedup ->
unique table + occurrence CSR) over one synthetic proteome already resident in
HBM.  Default workload at N=1: the SwissProt-scale FASTA the metric is quoted
on (BASELINE.json configs[2] "SwissProt (~560k proteins), trypsin, 2 missed
cleavages", which fits one MI355X) as a seeded synthetic proteome (SURVEY.md
§8(d), seed 3).  --config human is configs[1] (20k proteins, seed 2).
N>1 (torchrun, one rank per GPU): every rank builds its own protein shard of
the same size (seed + 1000*rank) -> weak scaling, no data-path collective.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--config swissprot|human|1k]
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

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BASELINE_METRIC = "peptides indexed/sec + mass-window queries/sec, SwissProt-scale FASTA"
WORKLOADS = {
    "human": ("UniProt-human-scale synthetic proteome (20,000 proteins, seed 2), trypsin, "
              "2 missed cleavages, 500-6000 Da MH+ (BASELINE.json configs[1])", 2),
    "1k": ("1k-protein synthetic proteome (seed 1), trypsin, 0 missed cleavages (configs[0])", 0),
    "swissprot": ("SwissProt-scale synthetic proteome (560,000 proteins, seed 3), trypsin, "
                  "2 missed cleavages (configs[2], single GPU)", 2),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="swissprot", choices=sorted(WORKLOADS))
    ap.add_argument("--queries", type=int, default=1_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    from dbindex_amd import fasta
    from dbindex_amd._native import DeviceBuffer, synchronize
    from dbindex_amd.engine import Engine
    from dbindex_amd.params import DBIndexSearchParams

    dist = None
    if world > 1:
        # coordination only (barrier, max time, sum of counts): the shards are
        # independent, so there is no data-path collective; gloo keeps torch's
        # own HIP runtime out of this process (see dbindex_amd/_native.py)
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    dev = local_rank

    desc, missed = WORKLOADS[args.config]
    base = dict(fasta.CONFIGS[args.config])
    base["seed"] = base["seed"] + 1000 * rank  # each rank its own shard of equal size
    t0 = time.time()
    pp = fasta.synthetic(with_defs=False, **base)
    log(f"[rank {rank}] synthetic {args.config}: P={pp.n_proteins} R={pp.n_residues} ({time.time() - t0:.1f}s)")
    prm = DBIndexSearchParams.trypsin(missed)

    # inputs resident in HBM before the timed region
    d_res = DeviceBuffer.from_numpy(pp.residues, dev)
    d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), dev)
    synchronize(dev)

    eng = Engine(prm, device=dev)

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
    # (the first build is cold: count + emit; the second may grow the bounded
    # digest's reservation and run it twice: neither is a steady-state build)
    eng.set_timing(True)
    warm_acc = {}
    n_warm = max(args.warmup, 1)
    skip = min(2, n_warm - 1)
    for i in range(n_warm):
        st = step()
        if i >= skip:
            accumulate(warm_acc)
    synchronize(dev)
    dominant = max(warm_acc.items(), key=lambda kv: kv[1][0])[0] if warm_acc else ""

    # timed region: events only on the dominant kernel (each timed stage costs
    # a few us of dispatch overhead; the other stages run untimed)
    eng.set_timing(True, only=dominant)
    stage_acc = {}
    if world > 1:
        dist.barrier()
    synchronize(dev)
    t_start = time.perf_counter()
    n_total = 0
    for _ in range(args.steps):
        st = step()
        n_total += st.n_total
        accumulate(stage_acc)
    synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start

    # whole-job: units of all ranks / max time over ranks
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nt = torch.tensor([n_total], dtype=torch.float64)
        dist.all_reduce(nt, op=dist.ReduceOp.SUM)
        n_total_all = float(nt.item())
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

    def pmc_traffic(stage):
        """HBM bytes per launch of `stage` from the newest committed rocprofv3
        PMC summary of this workload (profiles/<round>_<config>_summary.json,
        tools/prof_summary.py: 2 x FETCH_SIZE + WRITE_SIZE), or (None, None)."""
        import glob
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{args.config}_summary.json")))
        for f in reversed(files):
            st = json.load(open(f)).get("stages", {}).get(stage, {})
            if "traffic_bytes" in st:
                return st["traffic_bytes"], os.path.relpath(f, ROOT)
        return None, None

    kernels = kernel_table(warm_acc, n_warm - skip)
    timed = kernel_table(stage_acc, args.steps)
    dom = timed[0] if timed else None
    build_alg = st.n_residues + 8.0 * (st.n_proteins + 1) + 48.0 * st.n_total

    # secondary: mass-window queries/sec on the built index (1M queries, +-20 ppm)
    qps = None
    if args.queries > 0:
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
        qps = dict(value=nq * reps / tq, unit="queries/s", queries=nq, tol_ppm=20.0,
                   avg_hits=hits / nq, index="the build above")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # reference-semantics CPU restatement (oracle/cpu_ref.cpp), single thread
        # like the reference; bounded sample of the same workload
        from oracle import cref
        sample = pp if args.config != "swissprot" else pp.slice(0, 40000)
        t1 = time.perf_counter()
        oix = cref.Index(prm.to_c(), sample.residues, sample.offsets)
        t1 = time.perf_counter() - t1
        cpu = dict(value=oix.n_total / t1, unit="peptides indexed/s", cores=1, kind="port",
                   sample=f"{sample.n_proteins} proteins / {sample.n_residues} residues of the same "
                          f"workload ({oix.n_total} peptides, {t1:.1f}s); host CPU: {cpu_model()}",
                   seconds=t1)

    traffic, traffic_src = pmc_traffic(dom["kernel"]) if dom else (None, None)
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded proteome, SwissProt residue frequencies; SURVEY.md §8(d))",
            "config": {
                "workload": desc,
                "proteins_per_gpu": pp.n_proteins,
                "residues_per_gpu": pp.n_residues,
                "peptides_per_step_per_gpu": st.n_total,
                "unique_peptides": st.n_unique,
                "mass_keys": st.n_keys,
                "parallelism": f"protein-sharded x{world}, shard-local index" if world > 1 else "single GPU",
                "n_bins": st.n_bins,
                "n_big_bins": st.n_big_bins,
            },
            "roofline": None if dom is None else {
                "bound": "hbm",
                "kernel": dom["kernel"],
                "achieved": dom["gbps"],
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": dom["gbps"] / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": dom["alg_bytes"],
                "avg_launch_ms": dom["avg_ms"],
            },
            "build_roofline": {
                "alg_bytes": build_alg,
                "formula": "R + 8(P+1) + 48N (SURVEY.md §8(d))",
                "achieved_gbps": build_alg / (ms_per_step * 1e-3) / 1e9,
                "frac": build_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS,
            },
            "kernels": kernels,
            "kernels_note": "per-kernel HIP events (dispatch-packet start/stop) over the warmup builds; "
                            "the roofline kernel is re-timed inside the timed region",
            "queries": qps,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
