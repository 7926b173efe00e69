#!/bin/bash
# SQ counters of the TrEMBL count / bucket-count kernels
set -u -o pipefail
OUT=gpurun_out/r04g; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY \
  --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --config trembl --steps 1 --warmup 1 --no-cpu-baseline > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
python3 tools/sq_summary.py $OUT/pmc_sq
python3 - <<'PY'
import csv, glob, collections
p = glob.glob('gpurun_out/r04g/pmc_sq/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(p)):
    agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in agg.items():
    if c.get('SQ_WAVES', 0) > 1000:
        print(k[:70], 'SALU/wave %.0f' % (c['SQ_INSTS_SALU'] / c['SQ_WAVES']), 'LDSwait/cycle %.2f' % (c['SQ_WAIT_INST_LDS'] / max(c['SQ_WAVE_CYCLES'], 1)))
PY
echo ALLDONE
