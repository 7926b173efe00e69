"""Localise a COUNT-mode disagreement between two builds of the library
(in-tree vs DBI_OLD_LIB) over the TrEMBL-scale synthetic proteome: count every
chunk with both, bisect a differing chunk down to single proteins, print them.

    DBI_OLD_LIB=dbindex_amd/exp/old.so python tools/count_diff.py [--chunks 48]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dbindex_amd import _native, fasta  # noqa: E402
from dbindex_amd.engine import Engine  # noqa: E402
from dbindex_amd.params import DBIndexSearchParams  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=48)
    ap.add_argument("--proteins", type=int, default=50_000_000)
    ap.add_argument("--layout", default="separate", choices=["separate", "bench"])
    a = ap.parse_args()
    prm = DBIndexSearchParams.non_specific(50)
    cp = prm.to_c()
    B = ctypes.CDLL(os.path.abspath(os.environ["DBI_OLD_LIB"]))
    P = ctypes.c_void_p
    B.dbi_open.argtypes = [P, ctypes.c_int, P]
    B.dbi_count.argtypes = [P, P, ctypes.c_uint64, P, ctypes.c_uint64, P, P]
    hB = P()
    assert B.dbi_open(ctypes.byref(cp), 0, ctypes.byref(hB)) == 0

    def count_b(d_res, n_res, d_off, n):
        t, d = ctypes.c_uint64(), ctypes.c_uint64()
        assert B.dbi_count(hB, P(d_res), n_res, P(d_off), n, ctypes.byref(t), ctypes.byref(d)) == 0
        return t.value

    eng = Engine(cp, 0)
    gen = Engine(cp, 0)  # generator (its buffers stay put while eng counts)
    tables = fasta.synth_tables()
    seed = 4
    base = fasta.synth_residue_base(seed, 0, tables[0])
    CH = 1 << 20
    res_pos = 0
    found = []
    if a.layout == "bench":
        # bench.py run_trembl's layout: every chunk back to back in one buffer
        P_ = min(a.proteins, a.chunks * CH)
        lens = sum(int(fasta.synth_lengths(seed, q, min(CH, P_ - q), tables[0]).sum()) for q in range(0, P_, CH))
        d_all = _native.DeviceBuffer(lens + 16, 0)
        o_all = _native.DeviceBuffer(8 * (P_ + (P_ + CH - 1) // CH + 1), 0)
        chunks, rp, op = [], 0, 0
        for q in range(0, P_, CH):
            n = min(CH, P_ - q)
            d_res, d_off, n_res = gen.synth_proteome(seed, q, n, base + rp, tables)
            d_all.copy_from_device(rp, d_res, n_res)
            o_all.copy_from_device(8 * op, d_off, 8 * (n + 1))
            chunks.append((d_all.ptr + rp, n_res, o_all.ptr + 8 * op, n))
            rp += n_res
            op += n + 1
        _native.synchronize(0)
        ta = tb = ta2 = 0
        for ci, c in enumerate(chunks):
            x = eng.count_device(*c)[0]
            x2 = eng.count_device(*c)[0]
            y = count_b(*c)
            ta, ta2, tb = ta + x, ta2 + x2, tb + y
            print(json.dumps({"chunk": ci, "new": x, "new_again": x2, "old": y}), flush=True)
        print(json.dumps({"total_new": ta, "total_new_again": ta2, "total_old": tb}), flush=True)
        return
    for ci, p0 in enumerate(range(0, min(a.proteins, a.chunks * CH), CH)):
        n = min(CH, a.proteins - p0)
        d_res, d_off, n_res = gen.synth_proteome(seed, p0, n, base + res_pos, tables)
        res_pos += n_res
        ca = eng.count_device(d_res, n_res, d_off, n)[0]
        cb = count_b(d_res, n_res, d_off, n)
        print(json.dumps({"chunk": ci, "p0": p0, "new": ca, "old": cb}), flush=True)
        if ca == cb:
            continue
        off = np.zeros(n + 1, np.uint64)
        _native.check(_native.lib().dbi_dev_copy_d2h(0, off.ctypes.data_as(P), P(d_off), 8 * (n + 1)))
        res = np.zeros(n_res, np.uint8)
        _native.check(_native.lib().dbi_dev_copy_d2h(0, res.ctypes.data_as(P), P(d_res), n_res))

        def sub_counts(lo, hi):
            r = res[int(off[lo]):int(off[hi])]
            o = (off[lo:hi + 1] - off[lo]).astype(np.uint64)
            dr = _native.DeviceBuffer.from_numpy(np.concatenate([r, np.zeros(16, np.uint8)]), 0)
            do = _native.DeviceBuffer.from_numpy(o, 0)
            x = eng.count_device(dr.ptr, r.shape[0], do.ptr, hi - lo)[0]
            y = count_b(dr.ptr, r.shape[0], do.ptr, hi - lo)
            return x, y

        stack = [(0, n)]
        while stack:
            lo, hi = stack.pop()
            x, y = sub_counts(lo, hi)
            if x == y:
                continue
            if hi - lo == 1:
                seq = res[int(off[lo]):int(off[hi])].tobytes().decode("ascii")
                found.append({"protein": p0 + lo, "new": x, "old": y, "seq": seq})
                print(json.dumps(found[-1]), flush=True)
                continue
            mid = (lo + hi) // 2
            stack += [(lo, mid), (mid, hi)]
        if len(found) >= 8:
            break
    print(json.dumps({"found": len(found)}), flush=True)


if __name__ == "__main__":
    main()
