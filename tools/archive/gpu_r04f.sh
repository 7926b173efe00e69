#!/bin/bash
# bucket-count fast path: parity tests, then the TrEMBL bench line
set -u -o pipefail
OUT=gpurun_out/${TAG:-r04f}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -k "bucket or trembl or count" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 600 python bench.py --config trembl --steps 3 --warmup 3 > $OUT/trembl.json 2> $OUT/trembl.err || { tail -20 $OUT/trembl.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/trembl.json')); print('trembl', d['ms_per_step'], d['count_only']['ms'], d['cpu_baseline']['sample_bucket_parity'])"
echo ALLDONE
