#!/bin/bash
# giant fallback LDS path: giant / collision parity tests, then the semi-tryptic kernel trace
set -u -o pipefail
OUT=gpurun_out/${TAG:-r04fb}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -k "giant or semi_slice or collision or isobaric" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
bash tools/gpu_round.sh $(basename $OUT) prof_semi > $OUT/prof.out 2>&1 || { tail -20 $OUT/prof.out; exit 1; }
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$OUT/prof_semi/run_kernel_trace.csv")))
t = collections.defaultdict(list)
for r in rows:
    t[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(t.items(), key=lambda x: -sum(x[1]))[:16]:
    print(f"{sum(v)/len(v):8.3f} ms x{len(v):3d} {k}")
PY
echo ALLDONE
