#!/usr/bin/env python3
"""tools/ab_table.py DIR NAME... -- one line per bench log DIR/NAME.log: the
step time and the per-kernel times of the build (A/B runs on one box)."""
import json
import sys


def main():
    d = sys.argv[1]
    for name in sys.argv[2:]:
        line = open(f"{d}/{name}.log").read().strip().splitlines()[-1]
        b = json.loads(line)
        ks = {k["kernel"]: k["ms_per_build"] for k in b.get("kernels", [])}
        top = " ".join(f"{k}={ks[k]:.3f}" for k in ("digest", "chunk_sort", "finalize", "bin_scatter",
                                                     "chunk_sort_big", "chunk_sort_mid") if k in ks)
        print(f"{name:8s} ms/step {b['ms_per_step']:.4f}  {top}")


if __name__ == "__main__":
    main()
