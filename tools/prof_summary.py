#!/usr/bin/env python3
"""Summarise a gpu_round.sh profile directory into profiles/:

    python tools/prof_summary.py gpurun_out/<TAG> profiles/<round>_<config>

Writes <out>_kernel_stats.csv (the rocprofv3 --kernel-trace --stats summary,
copied verbatim), and <out>_summary.json: per build stage the average kernel
duration (rocprofv3) and the HBM traffic per launch from the separate PMC
passes, corrected as MI355X_MICROARCH.md prescribes for gfx950:
traffic = 2 x FETCH_SIZE (reads are tallied at half their bytes) + WRITE_SIZE,
both reported by rocprofv3 in KiB.
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
    ("void dbi::k_chunk_sort_list<512, 1984, false>", "chunk_sort_mid"),
    ("void dbi::k_chunk_sort_list<1024, 7936, true>", "chunk_sort_big"),
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
    ("k_digest_bounded", "digest"),
    ("k_synth_", "synth"),
    ("k_qroute", "query_route"),
    ("k_query_pairs", "query"),
    ("k_qcombine", "query"),
]


def stage_of(name: str) -> str:
    for sub, st in CONTAINS:
        if sub in name:
            return st
    for pre, st in STAGES:
        if name.startswith(pre):
            return st
    return name.split("(")[0]


def main(src: str, out: str) -> None:
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    stats_csv = os.path.join(src, "prof", "run_kernel_stats.csv")
    summary = {"source": src, "stages": {}}
    if os.path.exists(stats_csv):
        shutil.copyfile(stats_csv, out + "_kernel_stats.csv")
        for r in csv.DictReader(open(stats_csv)):
            st = summary["stages"].setdefault(stage_of(r["Name"]), {"calls": 0, "total_ns": 0.0})
            st["calls"] += int(r["Calls"])
            st["total_ns"] += float(r["TotalDurationNs"])
        for st in summary["stages"].values():
            st["avg_us"] = st["total_ns"] / st["calls"] / 1e3
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub, ctr in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == ctr:
                pmc[stage_of(r["Kernel_Name"])][ctr].append(float(r["Counter_Value"]) * 1024.0)
    for stage, d in pmc.items():
        st = summary["stages"].setdefault(stage, {})
        fetch = sum(d["FETCH_SIZE"]) / max(len(d["FETCH_SIZE"]), 1)
        write = sum(d["WRITE_SIZE"]) / max(len(d["WRITE_SIZE"]), 1)
        st["fetch_bytes_raw"] = fetch
        st["write_bytes"] = write
        st["traffic_bytes"] = 2.0 * fetch + write
    with open(out + "_summary.json", "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)
    for k, v in sorted(summary["stages"].items(), key=lambda kv: -kv[1].get("total_ns", 0)):
        print(f"{k:18s} avg {v.get('avg_us', 0):9.1f} us  traffic/launch {v.get('traffic_bytes', 0) / 1e6:9.1f} MB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
