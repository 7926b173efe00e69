"""CPU model of the chunking of a warm SwissProt build:
depth bins (k_depth_sample / k_depth_table / k_depth_chunks) against the radix
tail's 2^23 linear fine bins (k_chunk_bounds), from the oracle's index of the
same proteome.  Prints, per policy, the chunk-size classes that decide which
chunk-sort tier runs: main (<= 1984 records), big (1985-7936), and inside the
main chunks the records in bins of <= 64 (ranked), 65-512 (wave sorts) and
above 512 (mid tier).

    python tools/depth_sim.py [--config swissprot] [--sub-bits 20] [--bins-log2 16] [--T 1536]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CAP, BIG_CAP, RANK_MAX, WAVE_MAX = 1984, 7936, 64, 512


def bin_of(m, lo, hi, n):
    x = (m - lo) * (n / (hi - lo))
    return np.clip(np.where(x > 0, x, 0), 0, n - 1).astype(np.int64)


def load(config: str, cache: str):
    if os.path.exists(cache):
        z = np.load(cache)
        return z["mass"], z["cnt"], float(z["lo"]), float(z["hi"])
    from dbindex_amd import fasta
    from dbindex_amd.params import DBIndexSearchParams
    from oracle import cref
    pp = fasta.config(config)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    t = time.time()
    ix = cref.Index(cp, pp.residues, pp.offsets)
    u = ix.unique()
    mass = u["mass"]
    cnt = np.diff(u["occ_off"]).astype(np.int64)
    print(f"oracle index {time.time() - t:.1f} s: {mass.size} uniques, {cnt.sum()} records", flush=True)
    np.savez(cache, mass=mass, cnt=cnt, lo=cp.min_mh, hi=cp.max_mh)
    return mass, cnt, float(cp.min_mh), float(cp.max_mh)


def chunk_stats(name, sizes_main, bins_in_main, big_sizes, nchunks, extra=""):
    """bins_in_main: sizes of the (local or fine) bins inside the main-tier chunks."""
    b = np.asarray(bins_in_main)
    tot = b.sum()
    r_rank = b[b <= RANK_MAX].sum() / tot
    r_wave = b[(b > RANK_MAX) & (b <= WAVE_MAX)].sum() / tot
    r_mid = b[b > WAVE_MAX].sum() / tot
    big = np.asarray(big_sizes)
    print(f"{name}: chunks {nchunks} main {len(sizes_main)} (mean {np.mean(sizes_main):.0f}) big {big.size} "
          f"({big.sum() / 1e6:.2f} M recs, >3968: {(big > 3968).sum()}, >{BIG_CAP}: {(big > BIG_CAP).sum()}) | "
          f"main recs in bins <=64 {r_rank:.3f} 65-512 {r_wave:.3f} >512 {r_mid:.3f} (n>512 bins {(b > WAVE_MAX).sum()}) {extra}")


def radix_model(mass, cnt, T, fine_log2=23):
    lo, hi = mass[0], mass[-1]
    fb = bin_of(mass, lo, np.nextafter(hi, np.inf), 1 << fine_log2)
    fsz = np.bincount(fb, weights=cnt, minlength=1 << fine_log2).astype(np.int64)
    nz = np.nonzero(fsz)[0]
    starts = np.concatenate([[0], np.cumsum(fsz[nz])])  # start of each non-empty fine bin
    n = starts[-1]
    nch = (n + T - 1) // T
    # chunk 2c: fine bins starting in [cT, (c+1)T) minus a straddling bin > 512 -> chunk 2c+1
    main, big, inner = [], [], []
    sizes = fsz[nz]
    bstart = starts[:-1]
    idx = np.searchsorted(bstart, np.arange(nch + 1) * T, side="left")
    for c in range(nch):
        a, e = idx[c], idx[c + 1]
        if a >= e:
            continue
        s = sizes[a:e]
        # the last bin straddling (c+1)T and > 512: its own chunk
        last_end = bstart[e - 1] + s[-1]
        if s[-1] > WAVE_MAX and last_end > (c + 1) * T:
            m1 = s[-1]
            s = s[:-1]
            if m1 > CAP:
                big.append(m1)
            else:
                inner.append(m1)  # straddling bin: mid tier (counted as a >512 bin)
        if s.size:
            m = s.sum()
            if m > CAP:
                big.append(m)
            else:
                main.append(m)
                inner.extend(s.tolist())
    chunk_stats(f"radix 2^{fine_log2}", main, inner, big, 2 * nch)


def depth_model(mass, cnt, plo, phi, T, sub_bits, B, ns=1 << 19, local_log2=10, sample="uniq", alpha=0.0):
    """sample: "uniq" = ns evenly spaced uniques weighted by their counts (k_depth_sample);
    "rec" = ns evenly spaced records, weight 1.  alpha > 0: a sub-bin whose sampled weight
    exceeds alpha x the mean bin weight gets a bin of its own (the table's heavy isolation)."""
    nu = mass.size
    nsub = 1 << sub_bits
    nbins = 1 << B
    if sample == "uniq":
        j = (np.arange(ns, dtype=np.int64) * nu) // ns
        w = cnt[j]
    else:
        off = np.concatenate([[0], np.cumsum(cnt)])
        r = (np.arange(ns, dtype=np.int64) * off[-1]) // ns
        j = np.searchsorted(off, r, side="right") - 1
        w = np.ones(ns, np.int64)
    sb = bin_of(mass[j], plo, phi, nsub)
    hist = np.bincount(sb, weights=w, minlength=nsub).astype(np.int64)
    pre = np.concatenate([[0], np.cumsum(hist)[:-1]])
    tot = hist.sum()
    if alpha > 0:
        heavy = hist > alpha * tot / nbins
        H = int(heavy.sum())
        hb = np.concatenate([[0], np.cumsum(heavy)[:-1]])  # heavies before s
        nb2 = max(nbins - 2 * H, nbins // 2)
        tab = np.minimum(pre * nb2 // tot + 2 * hb + heavy, nbins - 1)
    else:
        H = 0
        tab = np.minimum(pre * nbins // tot, nbins - 1)
    db = tab[bin_of(mass, plo, phi, nsub)]
    bsz = np.bincount(db, weights=cnt, minlength=nbins).astype(np.int64)
    bstart = np.concatenate([[0], np.cumsum(bsz)])
    n = bstart[-1]
    nch = (n + T - 1) // T
    # first_ge(x): first b with bstart[b] >= x
    fg = lambda x: np.searchsorted(bstart, x, side="left")
    main, big, inner, pair_split = [], [], [], 0
    # record-level local bins need the masses per chunk: masses sorted already
    rec_m = np.repeat(mass, cnt)
    xb = rec_m.view(np.uint64) >> np.uint64(8)
    nl = 1 << local_log2
    pair_work = []
    for c in range(nch):
        s0 = bstart[fg(min(c * T, n))]
        j1 = fg(min((c + 1) * T, n))
        s1 = bstart[j1]
        split = s1
        if s1 - s0 > CAP and j1 > 0 and bstart[j1 - 1] > s0:
            split = bstart[j1 - 1]
        w = 0
        for a, e in ((s0, split), (split, s1)):
            m = e - a
            if m == 0:
                continue
            if e == s1 and a == split and split != s1:
                pair_split += 1
            if m > CAP:
                big.append(m)
                continue
            main.append(m)
            w += m
            x = xb[a:e]
            mn, mx = int(x.min()), int(x.max())
            scale = nl / (float(mx - mn) + 1.0)
            lb = np.minimum(((x - np.uint64(mn)).astype(np.float64) * scale).astype(np.int64), nl - 1)
            inner.extend(np.bincount(lb)[np.bincount(lb) > 0].tolist())
        pair_work.append(w)
    pw = np.asarray(pair_work)
    chunk_stats(f"depth sub2^{sub_bits} B{B} T{T} {sample} a{alpha} H{H} local2^{local_log2}", main, inner, big, 2 * nch,
                f"| split pairs {pair_split}, pair recs p50 {np.median(pw):.0f} p99 {np.percentile(pw, 99):.0f} max {pw.max()}"
                f" | depth bins > {CAP}: {(bsz > CAP).sum()}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="swissprot")
    ap.add_argument("--cache", default="/tmp/depth_sim_{}.npz")
    ap.add_argument("--sub-bits", type=int, nargs="*", default=[20])
    ap.add_argument("--bins-log2", type=int, nargs="*", default=[16])
    ap.add_argument("--T", type=int, nargs="*", default=[1536])
    ap.add_argument("--radix", action="store_true")
    ap.add_argument("--sample", nargs="*", default=["uniq"])
    ap.add_argument("--alpha", type=float, nargs="*", default=[0.0])
    ap.add_argument("--local-log2", type=int, nargs="*", default=[10])
    a = ap.parse_args()
    mass, cnt, plo, phi = load(a.config, a.cache.format(a.config))
    for T in a.T:
        if a.radix:
            radix_model(mass, cnt, T)
        for sb in a.sub_bits:
            for B in a.bins_log2:
                for smp in a.sample:
                    for al in a.alpha:
                        for ll in a.local_log2:
                            depth_model(mass, cnt, plo, phi, T, sb, B, sample=smp, alpha=al, local_log2=ll)


if __name__ == "__main__":
    main()
