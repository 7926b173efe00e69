"""Per-kernel averages of a rocprofv3 --pmc SQ pass (tools/gpu_round.sh pmc_sq):
VALU instructions per wave, the share of wave cycles spent waiting, LDS bank
conflicts per LDS instruction.   python tools/sq_summary.py gpurun_out/TAG/pmc_sq"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "."
path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(path)):
    agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(agg.items(), key=lambda kv: -sum(kv[1].get("SQ_WAVE_CYCLES", [0]))):
    a = {n: sum(v) / len(v) for n, v in c.items()}
    if a.get("SQ_WAVES", 0) < 1000:
        continue
    w = a["SQ_WAVES"]
    print(f"{k[:60]:60s} waves {w:9.0f}  VALU/wave {a['SQ_INSTS_VALU'] / w:7.0f}  LDS/wave {a['SQ_INSTS_LDS'] / w:6.0f}  "
          f"wait {a['SQ_WAIT_ANY'] / a['SQ_WAVE_CYCLES']:.2f}  conflicts/LDS {a['SQ_LDS_BANK_CONFLICT'] / max(a['SQ_INSTS_LDS'], 1):.2f}")
