#!/usr/bin/env python3
"""Summarise a gpu_round.sh profile directory into profiles/:

    python tools/prof_summary.py gpurun_out/<TAG> profiles/<round>_<config>

Writes <out>_kernel_stats.csv (the rocprofv3 --kernel-trace --stats summary,
copied verbatim), and <out>_summary.json: per build stage the average kernel
duration (rocprofv3) and the HBM traffic per launch from the separate PMC
passes, corrected as MI355X_MICROARCH.md prescribes for gfx950:
traffic = 2 x FETCH_SIZE (reads are tallied at half their bytes) + WRITE_SIZE,
both reported by rocprofv3 in KiB.

Degenerate launches -- a stage's launch far below that stage's median
(< DEGENERATE x median: the empty tail of a build whose digest outgrew its
reservation and was redone, an empty list grid) -- are left out of the
per-launch averages (duration from the per-dispatch kernel trace, traffic
from the per-dispatch counters) and counted in `dropped_launches`.  The
`build` entry sums the build's own stages (launches per build x the average
per launch): its device time and its PMC traffic, next to SURVEY.md §8(d)'s
algorithmic bytes when the bench line of the same workload is given.
"""
from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys

# rocprof kernel name prefix -> bench/engine stage name
STAGES = [
    ("dbi::k_tile_proteins", "tile_proteins"),
    ("void dbi::k_digest_fused<", "digest"),
    ("dbi::k_digest_bounded", "digest"),
    ("dbi::k_digest_count_cuts", "digest_count"),
    ("void dbi::k_digest<false", "digest_count"),
    ("void dbi::k_digest<true", "digest_emit"),
    ("void dbi::k_radix_hist<", "radix_hist"),
    ("void dbi::k_radix_scatter<", "radix_scatter"),
    ("dbi::k_chunk_bounds", "chunk_bounds"),
    ("void dbi::k_chunk_sort<", "chunk_sort"),
    ("dbi::k_chunk_sort_big", "chunk_sort_big"),
    ("void dbi::k_bin_sort_mid<", "chunk_sort_mid"),
    ("void dbi::k_chunk_sort_list<512, 1984, false>", "chunk_sort_mid"),  # rounds 2-3
    ("void dbi::k_chunk_sort_list<1024, 7936", "chunk_sort_big"),
    ("dbi::k_big_chunks", "chunk_sort_giant"),
    ("dbi::k_finalize", "finalize"),
    ("dbi::k_key_flags", "key_flags"),
    ("dbi::k_write_tail", "write_tail"),
    ("dbi::k_scan", "scan"),
    ("dbi::k_off64_to_32", "off64_to_32"),
    ("dbi::k_query", "query"),
]


# substrings checked first (template arguments tell the stages apart)
CONTAINS = [
    ("OwnerDigit", "owner_partition"),
    ("PairDigit", "query_route"),
    ("k_giant_", "chunk_sort_giant"),
    ("k_finalize", "finalize"),  # k_finalize<NT, ITEMS> since round 4
    ("k_radix_hist_u8", "radix_hist_u8"),
    ("k_chunk_sort_list<512, 3968", "chunk_sort_big"),  # the big tier's smaller size class
    ("k_digest_bounded", "digest"),
    ("k_digest_count_cuts", "digest_count"),
    ("k_synth_", "synth"),
    ("k_qroute", "query_route"),
    ("k_query_pairs", "query"),
    ("k_qcombine", "query"),
    ("k_part_scatter", "bin_scatter"),  # depth bins (round 5)
    ("k_part_hist", "part_hist"),
    ("k_part_plan", "part_plan"),
    ("k_depth_sample", "depth_map"),
    ("k_depth_table", "depth_map"),
    ("k_depth_starts", "chunk_bounds"),
    ("k_depth_chunks", "chunk_bounds"),
]


def stage_of(name: str) -> str:
    for sub, st in CONTAINS:
        if sub in name:
            return st
    for pre, st in STAGES:
        if name.startswith(pre):
            return st
    return name.split("(")[0]


DEGENERATE = 0.1
# not part of a warm build: the bench's copy probe, the runtime's own blits,
# the cold build's count / emit digest
NOT_BUILD = ("dbi::k_hbm_copy", "__amd_rocclr", "digest_count", "digest_emit")


def _keep(vals):
    """Indices of the non-degenerate values of one stage."""
    if len(vals) < 3:
        return list(range(len(vals)))
    med = sorted(vals)[len(vals) // 2]
    return [i for i, v in enumerate(vals) if v >= DEGENERATE * med]


def main(src: str, out: str, bench_json: str = "") -> None:
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    stats_csv = os.path.join(src, "prof", "run_kernel_stats.csv")
    trace_csv = os.path.join(src, "prof", "run_kernel_trace.csv")
    summary = {"source": src, "degenerate_below_median_frac": DEGENERATE, "stages": {}}
    if os.path.exists(stats_csv):
        shutil.copyfile(stats_csv, out + "_kernel_stats.csv")
        for r in csv.DictReader(open(stats_csv)):
            st = summary["stages"].setdefault(stage_of(r["Name"]), {"calls": 0, "total_ns": 0.0})
            st["calls"] += int(r["Calls"])
            st["total_ns"] += float(r["TotalDurationNs"])
        for st in summary["stages"].values():
            st["avg_us_all"] = st["total_ns"] / st["calls"] / 1e3
    if os.path.exists(trace_csv):
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(trace_csv)):
            durs[stage_of(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for stage, d in durs.items():
            keep = _keep(d)
            st = summary["stages"].setdefault(stage, {})
            st["launches"] = len(d)
            st["dropped_launches"] = len(d) - len(keep)
            st["avg_us"] = sum(d[i] for i in keep) / max(len(keep), 1)
    for st in summary["stages"].values():  # no trace: the stats' average
        if "avg_us" not in st and "avg_us_all" in st:
            st["avg_us"] = st["avg_us_all"]
    pmc = collections.defaultdict(lambda: collections.defaultdict(dict))
    for sub, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == ctr:
                k = stage_of(r["Kernel_Name"])
                pmc[k][ctr][int(r["Dispatch_Id"])] = float(r["Counter_Value"]) * 1024.0
    builds_pmc = 0
    for stage, d in pmc.items():
        st = summary["stages"].setdefault(stage, {})
        f = [d["FETCH_SIZE"][k] for k in sorted(d["FETCH_SIZE"])]
        w = [d["WRITE_SIZE"][k] for k in sorted(d["WRITE_SIZE"])]
        kf, kw = _keep([2 * x for x in f]), _keep(w)
        fetch = sum(f[i] for i in kf) / max(len(kf), 1)
        write = sum(w[i] for i in kw) / max(len(kw), 1)
        st["fetch_bytes_raw"] = fetch
        st["write_bytes"] = write
        st["traffic_bytes"] = 2.0 * fetch + write
        st["pmc_launches"] = len(kw)
        if stage == "finalize":
            builds_pmc = len(kw)
    # one build = one finalize launch
    fin = summary["stages"].get("finalize", {})
    builds_trace = fin.get("launches", 0) - fin.get("dropped_launches", 0)
    build = {"stages": {}, "device_ms": 0.0, "traffic_bytes": 0.0}
    for stage, st in summary["stages"].items():
        if any(stage.startswith(x) for x in NOT_BUILD):
            continue
        # launches per build (0: a stage of the few builds that took another
        # path -- the cold build, the first warm build -- not of the steady state)
        per = None
        if builds_trace and "launches" in st:
            per = round((st["launches"] - st.get("dropped_launches", 0)) / builds_trace)
            build["device_ms"] += per * st["avg_us"] / 1e3
        if builds_pmc and "traffic_bytes" in st:
            per_p = per if per is not None else round(st["pmc_launches"] / builds_pmc)
            build["traffic_bytes"] += per_p * st["traffic_bytes"]
            per = per if per is not None else per_p
        if per:
            build["stages"][stage] = per
    build["builds_in_trace"] = builds_trace
    build["builds_in_pmc"] = builds_pmc
    if bench_json and os.path.exists(bench_json):
        line = json.load(open(bench_json))
        cfg = line.get("config", {})
        br = line.get("build_roofline") or (line.get("roofline") or {})
        alg = br.get("alg_bytes") or br.get("alg_bytes_per_build")
        if alg:
            build["alg_bytes"] = alg
            build["traffic_over_alg"] = build["traffic_bytes"] / alg if build["traffic_bytes"] else None
        build["bench_ms_per_step"] = line.get("ms_per_step")
        build["workload"] = cfg.get("workload")
    summary["build"] = build
    with open(out + "_summary.json", "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    for k, v in sorted(summary["stages"].items(), key=lambda kv: -kv[1].get("total_ns", 0)):
        print(f"{k:18s} avg {v.get('avg_us', 0):9.1f} us ({v.get('dropped_launches', 0)} degenerate dropped)  "
              f"traffic/launch {v.get('traffic_bytes', 0) / 1e6:9.1f} MB")
    print(f"build: {build['device_ms']:.3f} ms device, {build['traffic_bytes'] / 1e9:.3f} GB PMC traffic"
          + (f", {build['alg_bytes'] / 1e9:.3f} GB algorithmic ({build['traffic_over_alg']:.2f}x)"
             if build.get("alg_bytes") and build.get("traffic_over_alg") else ""))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
