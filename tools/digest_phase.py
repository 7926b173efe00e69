#!/usr/bin/env python3
"""Phase clocks of the partitioning digest (experiment build with
-DDBI_DIGEST_CLOCK, e.g. tools/exp/dclock.so via DBI_LIB_PATH): warm SwissProt
builds, then the summed s_memtime cycles of thread 0 of every staged tile
between the kernel's barriers -- bit maps / compaction + balance / slot
bounds + reservation / walks / record rebuild / partition -- per tile.
Results of a clock build are valid (the clocks only read a counter)."""
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from dbindex_amd import _native, fasta  # noqa: E402
from dbindex_amd.engine import Engine  # noqa: E402
from dbindex_amd.params import DBIndexSearchParams  # noqa: E402

NAMES = ["load + bit maps", "compaction + balance", "slot bounds + reserve", "walks", "record rebuild",
         "partition"]


def main():
    pp = fasta.config(sys.argv[1] if len(sys.argv) > 1 else "swissprot")
    L = _native.lib()
    fn = L.dbi_debug_digest_clock
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    d_res = _native.DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), 0)
    d_off = _native.DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), 0)
    buf = (ctypes.c_ulonglong * 16)()
    with Engine(DBIndexSearchParams.trypsin(2).to_c(), 0) as eng:
        eng.set_timing(False)
        for _ in range(4):
            eng.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)
        fn(buf, 1)
        reps = 5
        for _ in range(reps):
            eng.build_device(d_res.ptr, pp.n_residues, d_off.ptr, pp.n_proteins)
        _native.synchronize(0)
        fn(buf, 0)
    v = list(buf)
    tiles = v[8] or 1
    tot = sum(v[:6])
    out = dict(staged_tiles_per_build=tiles / reps, slots_per_tile=v[9] / tiles, candidates_per_tile=v[10] / tiles,
               phases={n: dict(cycles_per_tile=v[k] / tiles, share=v[k] / tot if tot else 0.0)
                       for k, n in enumerate(NAMES)},
               partition={n: dict(cycles_per_tile=v[11 + k] / tiles, share=v[11 + k] / tot if tot else 0.0)
                          for k, n in enumerate(["bins + ranks", "scan + region reservation",
                                                 "restage in digit order", "runs written"])},
               bins_alone=dict(cycles_per_tile=v[15] / tiles, share=v[15] / tot if tot else 0.0))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
