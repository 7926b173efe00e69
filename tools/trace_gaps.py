"""Per-build span vs kernel time from a rocprofv3 kernel trace.

  python tools/trace_gaps.py gpurun_out/TAG/prof/run_kernel_trace.csv [--start tile_proteins]

A build starts at each dispatch whose kernel name contains --start (the
first kernel of a warm build) and runs to the dispatch before the next one.
For each build: the span (first start to last end), the summed kernel
durations, the idle time between them (launch / dependency gaps) and the
kernel count; then the medians over the builds.  On a launch-bound build
(the human config) the gaps are what a graph replay still pays per kernel.
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--start", default="tile_proteins")
    a = ap.parse_args()
    rows = []
    with open(a.trace, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    builds, cur = [], None
    for s, e, name in rows:
        if a.start in name:
            if cur:
                builds.append(cur)
            cur = []
        if cur is not None:
            cur.append((s, e, name))
    if cur:
        builds.append(cur)
    out = []
    for b in builds:
        span = (max(e for _, e, _ in b) - b[0][0]) / 1e3
        busy = sum(e - s for s, e, _ in b) / 1e3
        out.append({"kernels": len(b), "span_us": span, "kernel_us": busy, "gap_us": span - busy})
    if not out:
        print(json.dumps({"builds": 0}))
        return 1
    med = {k: statistics.median(o[k] for o in out) for k in ("kernels", "span_us", "kernel_us", "gap_us")}
    print(json.dumps({"builds": len(out), "median": med, "per_gap_us": med["gap_us"] / max(med["kernels"] - 1, 1)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
