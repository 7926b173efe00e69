#!/bin/bash
# largest-first wave sorts in k_chunk_sort: A/B against an experiment build without (dbindex_amd/exp/nolpt.so)
set -u -o pipefail
OUT=gpurun_out/${TAG:-r04lpt}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -k "swissprot_full or semi_slice or wide or collision or big_bins or isobaric or grids or synthetic" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for v in lpt nolpt lpt nolpt; do
  if [ $v = nolpt ]; then export DBI_LIB_PATH=dbindex_amd/exp/nolpt.so; else unset DBI_LIB_PATH; fi
  timeout -k 10 300 python bench.py --config swissprot --steps 20 --warmup 5 --no-cpu-baseline --queries 0 > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1])
print('$v', round(d['ms_per_step'],4), [(k['kernel'], round(k['ms_per_build'],4)) for k in d['kernels']][:7])"
done
echo ALLDONE
