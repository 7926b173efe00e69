#!/usr/bin/env python3
"""Phase clocks of the chunk sort (experiment build with -DDBI_PHASE_CLOCK,
e.g. tools/exp/pclock.so via DBI_LIB_PATH): warm builds of a bench config,
then the summed s_memtime cycles of thread 0 of every sort_chunk call between
its barriers -- load + runs / small-bin ranks / wave sorts of the wide bins /
block-level sorts (the big tier only) / finish (verification, heads, output)
-- for the main chunk sort and the big tier apart.  Results of a clock build
are valid (the clocks only read a counter).
  DBI_LIB_PATH=tools/exp/pclock.so python tools/chunk_phase.py [semi|swissprot]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import WORKLOADS  # noqa: E402
from dbindex_amd import _native, fasta  # noqa: E402
from dbindex_amd.engine import Engine  # noqa: E402

NAMES = ["load + runs", "small-bin ranks", "wave sorts", "block sorts", "finish"]


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "semi"
    _, proteome, make_params, _ = WORKLOADS[config]
    pp = fasta.synthetic(with_defs=False, **fasta.CONFIGS[proteome])
    L = _native.lib()
    fn = L.dbi_debug_phase_clock
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    d_res = _native.DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), 0)
    d_off = _native.DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), 0)
    buf = (ctypes.c_ulonglong * 48)()
    with Engine(make_params(), 0) as eng:
        eng.set_timing(False)
        for _ in range(3):
            eng.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)
        _native.synchronize(0)
        fn(buf, 1)
        reps = 2
        for _ in range(reps):
            eng.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)
        _native.synchronize(0)
        fn(buf, 0)
    v = list(buf)
    out = {}
    for name, base in (("chunk_sort", 0), ("big_tier", 16)):
        blocks = v[base + 8] or 1
        tot = sum(v[base:base + 5]) or 1
        out[name] = dict(calls_per_build=v[base + 8] / reps, records_per_build=v[base + 9] / reps,
                         records_per_call=v[base + 9] / blocks, wide_bins_per_call=v[base + 10] / blocks,
                         phases={n: dict(cycles_per_call=v[base + k] / blocks, share=v[base + k] / tot)
                                 for k, n in enumerate(NAMES)})
    # g[33..35]: wide bins of the big tier by block-level sort (tag counting sort / compact-key
    # network / full-key bitonic), g[37..39]: their cycles
    out["big_tier_block_sorts"] = {n: dict(bins_per_build=v[32 + k] / reps,
                                           cycles_per_bin=v[36 + k] / max(v[32 + k], 1))
                                   for k, n in ((1, "tag_sort"), (2, "compact_key"), (3, "bitonic"))}
    nb = max(sum(v[33:36]), 1)
    out["big_tier_distinct_masses"] = dict(mean_per_bin=v[40] / nb, share_le16=v[41] / nb, share_le256=v[42] / nb,
                                           max=v[43])
    out["wave_sorted_bins"] = {n: dict(per_build=v[44 + k] / reps, single_mass_share=v[46 + k] / max(v[44 + k], 1))
                               for k, n in ((0, "chunk_sort"), (1, "big_tier"))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
