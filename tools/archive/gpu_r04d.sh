#!/bin/bash
# round-4 GPU iteration: tests + shard budget, then A/B of the mid-tier bin split
# (prev = the previous commit's library) on swissprot and semi (+ notag on semi)
set -u -o pipefail
OUT=gpurun_out/r04d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=3 -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 200 python tools/shard_budget.py --reps 4 > $OUT/budget.json 2> $OUT/budget.err || { tail -20 $OUT/budget.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/budget.json')); print('budget', d['front_ms'], d['exchange_model_ms'], d['merge_max_ms'], d.get('fixed_ms'), d.get('model_ms'))"
bash tools/ab_variants.sh r04d/ab base prev wsl256 base:1792 base prev wsl256 || exit 1
AB_CONFIG=semi bash tools/ab_variants.sh r04d/ab_semi base env-DBI_SEMI_BOUNDED=0 notag prev || exit 1
echo ALLDONE
