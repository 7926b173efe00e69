#!/bin/bash
# device-sized warm shard digests: the sharded parity tests, then the one-rank general path (fixed costs)
set -u -o pipefail
OUT=gpurun_out/${TAG:-r04k}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -k "shard or scale" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 300 python tools/shard_budget.py --reps 4 > $OUT/budget.json 2> $OUT/budget.err || { tail -20 $OUT/budget.err; exit 1; }
python3 -c "
import json; s=open('$OUT/budget.json').read(); d=json.loads(s[s.index('{'):])
print('budget', d['front_ms'], d['exchange_model_ms'], d['merge_max_ms'], d.get('fixed_ms'), d.get('model_ms'), [round(x['fixed_ms'],3) for x in d['fixed_one_rank']])"
echo ALLDONE
