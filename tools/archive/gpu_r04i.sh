#!/bin/bash
# SQ counters + kernel trace of the semi-tryptic build (oversize chunk tiers)
set -u -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY \
  --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --config semi --steps 1 --warmup 2 --queries 0 --no-cpu-baseline > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
python3 tools/sq_summary.py $OUT/pmc_sq
python3 - <<'PY'
import csv, glob, collections
p = glob.glob('gpurun_out/r04i/pmc_sq/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(p)):
    k = r['Kernel_Name'].split('(')[0]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in agg.items():
    if c.get('SQ_WAVES', 0) > 1000:
        print(k[:70], 'SALU/wave %.0f' % (c['SQ_INSTS_SALU'] / c['SQ_WAVES']), 'LDSwait/cycle %.2f' % (c['SQ_WAIT_INST_LDS'] / max(c['SQ_WAVE_CYCLES'], 1)), 'cycles/wave %.0f' % (c['SQ_WAVE_CYCLES'] / c['SQ_WAVES']))
PY
echo ALLDONE
