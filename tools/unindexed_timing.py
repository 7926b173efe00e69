"""SEARCH_UNINDEXED timing: DBIndexer in SEARCH_UNINDEXED mode
over the synthetic SwissProt-scale proteome -- the one-off device digest of the
ProteinCache, then cutAndSearch latency for single 10-ppm ranges and for a
batch of 1000 ranges -- beside the CPU restatement re-cutting the proteome for
one search (what the reference does per search, DBIndexer.java:707-747).

    python tools/unindexed_timing.py [--config swissprot] [--mode resident|stream]
                                     [--enzyme trypsin|semi|nonspecific] [--cpu-proteins 20000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dbindex_amd import fasta  # noqa: E402
from dbindex_amd.indexer import DBIndexer, IndexerMode  # noqa: E402
from dbindex_amd.params import DBIndexSearchParams, tolerance_in_dalton  # noqa: E402
from dbindex_amd.store import MassRange, MassRangeFilteringIndexHip  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="swissprot")
    ap.add_argument("--cpu-proteins", type=int, default=20000)
    ap.add_argument("--mode", default="resident", choices=["resident", "stream"])
    ap.add_argument("--enzyme", default="trypsin", choices=["trypsin", "semi", "nonspecific"])
    ap.add_argument("--singles", type=int, default=200)
    ap.add_argument("--batch", type=int, default=1000)
    a = ap.parse_args()
    pp = fasta.config(a.config)
    prm = {"trypsin": lambda: DBIndexSearchParams.trypsin(2),
           "semi": lambda: DBIndexSearchParams.semi_tryptic(2),
           "nonspecific": lambda: DBIndexSearchParams.non_specific(50)}[a.enzyme]()
    mode = MassRangeFilteringIndexHip.STREAM if a.mode == "stream" else MassRangeFilteringIndexHip.RESIDENT
    t0 = time.perf_counter()
    ix = DBIndexer(prm, IndexerMode.SEARCH_UNINDEXED, indexStore=MassRangeFilteringIndexHip(prm, mode=mode))
    ix.init()
    ix.run(pp)
    t_cache = time.perf_counter() - t0
    rng = np.random.default_rng(3)
    masses = rng.uniform(800.0, 3500.0, max(a.batch, a.singles))
    # single-range searches (10 ppm)
    ts, n_hits = [], 0
    for m in masses[:a.singles]:
        t = time.perf_counter()
        r = ix.getSequencesUsingPPMTolerance(float(m), 10.0)
        ts.append(time.perf_counter() - t)
        n_hits += len(r)
    # one search with 1000 ranges
    ranges = [MassRange(float(m), tolerance_in_dalton(float(m), 10.0)) for m in masses[:a.batch]]
    t = time.perf_counter()
    rb = ix.getSequences(ranges)
    t_batch = time.perf_counter() - t
    out = {"config": a.config, "mode": a.mode, "enzyme": a.enzyme, "proteins": pp.n_proteins, "residues": pp.n_residues,
           "protein_cache_and_device_digest_s": round(t_cache, 4),
           "single_range_ms_median": round(1e3 * float(np.median(ts)), 4),
           "single_range_hits_mean": n_hits / len(ts),
           "batch_ranges": a.batch, "batch_ms": round(1e3 * t_batch, 3), "batch_hits": len(rb)}
    # CPU: the reference's per-search re-cut, on a bounded protein sample
    try:
        if a.cpu_proteins <= 0:
            raise RuntimeError("skipped")
        from oracle import cref
        sub = pp.slice(0, min(a.cpu_proteins, pp.n_proteins))
        t = time.perf_counter()
        cref.cut_and_search(prm.to_c(), sub.residues, sub.offsets, [float(masses[0])],
                            [tolerance_in_dalton(float(masses[0]), 10.0)])
        dt = time.perf_counter() - t
        out["cpu_recut_s_per_search_extrapolated"] = round(dt * pp.n_residues / max(sub.n_residues, 1), 4)
        out["cpu_sample_proteins"] = sub.n_proteins
    except Exception as e:  # the oracle is optional here
        out["cpu_error"] = str(e)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
