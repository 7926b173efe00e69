#!/bin/bash
# mid-tier size classes: the GPU suite, then bench lines (5 warmup builds) of swissprot / human / semi
set -u -o pipefail
OUT=gpurun_out/${TAG:-r04n}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for c in swissprot human semi; do
  steps=20; [ $c = semi ] && steps=8
  timeout -k 10 600 python bench.py --config $c --steps $steps --warmup 5 --queries 0 --no-cpu-baseline > $OUT/$c.json 2> $OUT/$c.err || { tail -20 $OUT/$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$c.json'))
print('$c', round(d['ms_per_step'],4), [(k['kernel'], round(k['ms_per_build'],4)) for k in d['kernels']][:9])"
done
echo ALLDONE
