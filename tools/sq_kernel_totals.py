"""Per-kernel totals of a rocprofv3 --pmc pass (SQ counters), as JSON: for each
kernel its launches and the summed counters (tools/gpu_round.sh pmc_sq_trembl;
bench.py's TrEMBL line reads SQ_INSTS_VALU of the bucket-count kernel from it
for the VALU issue roofline).
    python tools/sq_kernel_totals.py gpurun_out/TAG/trembl_sq > profiles/TAG_trembl_sq.json"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "."
path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
out = {k: dict(launches=len(disp[k]), **{n: v for n, v in c.items()}) for k, c in tot.items()}
print(json.dumps(dict(source=os.path.relpath(path, d), kernels=out), indent=1))
