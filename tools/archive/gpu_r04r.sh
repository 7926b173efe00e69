#!/bin/bash
# HBM traffic (FETCH / WRITE passes) of the semi-tryptic build's kernels
set -u -o pipefail
OUT=gpurun_out/r04r; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --config semi --steps 1 --warmup 2 --queries 0 --no-cpu-baseline > $OUT/f.log 2>&1 || { tail -20 $OUT/f.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --config semi --steps 1 --warmup 2 --queries 0 --no-cpu-baseline > $OUT/w.log 2>&1 || { tail -20 $OUT/w.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
res = {}
for kind in ('fetch', 'write'):
    p = glob.glob(f'gpurun_out/r04r/pmc_{kind}/**/*counter_collection.csv', recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        agg[r['Kernel_Name'].split('(')[0]].append(float(r['Counter_Value']))
    res[kind] = agg
for k in sorted(res['write'], key=lambda k: -sum(res['write'][k]))[:14]:
    f = res['fetch'].get(k, [0]); w = res['write'][k]
    print(f'{k[:60]:60s} n={len(w):3d} fetch/launch {sum(f)/max(len(f),1)/1e9:8.3f} GB(raw)  write/launch {sum(w)/len(w)/1e9:8.3f} GB')
PY
echo ALLDONE
