"""Fine-bin statistics of a built index: how the records fall into the 2^k
mass bins the chunk sort works on, and what a big bin holds.

  python tools/bin_stats.py [--config swissprot] [--bits 23]

Builds the config's proteome on the GPU, exports the unique table and the
occurrence CSR, and counts per fine bin (the engine's bin map over
[minMH, maxMH]): records (occurrences), distinct masses, unique peptides.
Prints one JSON object: the share of records in bins above 64 / 128 / 256 /
512 / 1984 / 7936 records, and for bins above 512 the percentiles of their
size, distinct masses and unique-peptide fraction (DESIGN.md §8 "Next").
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="swissprot")
    ap.add_argument("--bits", type=int, default=23)
    a = ap.parse_args()
    from dbindex_amd import fasta
    from dbindex_amd.engine import Engine
    from dbindex_amd.params import DBIndexSearchParams
    pp = fasta.config(a.config, with_defs=False)
    params = DBIndexSearchParams.trypsin(2)
    with Engine(params.to_c(), 0) as eng:
        eng.build(pp)
        ex = eng.export()
    mass = ex["mass"]
    occ = np.diff(ex["occ_off"]).astype(np.int64)  # records per unique peptide
    lo, hi = float(params.min_precursor_mass), float(params.max_precursor_mass)
    nb = 1 << a.bits
    b = np.clip(((mass - lo) * (nb / (hi - lo))).astype(np.int64), 0, nb - 1)  # unique table is mass-sorted
    recs = np.bincount(b, weights=occ, minlength=nb).astype(np.int64)
    uniq = np.bincount(b, minlength=nb)
    newm = np.r_[True, mass[1:] != mass[:-1]] | np.r_[True, b[1:] != b[:-1]]
    dmass = np.bincount(b, weights=newm, minlength=nb).astype(np.int64)
    total = int(recs.sum())
    out = {"config": a.config, "bins": nb, "records": total, "unique": int(mass.shape[0]), "share_above": {}}
    for th in (64, 128, 256, 512, 1984, 7936):
        m = recs > th
        out["share_above"][str(th)] = {"bins": int(m.sum()), "records": int(recs[m].sum()),
                                       "fraction": float(recs[m].sum() / max(total, 1))}
    big = recs > 512
    if big.any():
        q = [10, 50, 90, 99, 100]
        out["bins_above_512"] = {
            "percentiles": q,
            "records": [float(x) for x in np.percentile(recs[big], q)],
            "distinct_masses": [float(x) for x in np.percentile(dmass[big], q)],
            "unique_fraction": [float(x) for x in np.percentile(uniq[big] / recs[big], q)],
        }
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
