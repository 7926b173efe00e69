#!/bin/bash
# round-4 GPU iteration: tests [+ budget] (A), or benches + tag-sort A/B (B)
set -u -o pipefail
PART=${1:-A}; OUT=gpurun_out/r04c; mkdir -p $OUT
if [ "$PART" = A ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=3 -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
  tail -1 $OUT/t.log
  timeout -k 10 250 python tools/shard_budget.py --reps 4 > $OUT/budget.json 2> $OUT/budget.err || { tail -20 $OUT/budget.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/budget.json')); print('budget', d['front_ms'], d['exchange_model_ms'], d['merge_max_ms'], d.get('fixed_ms'), d.get('model_ms'))"
else
  for c in swissprot human trembl semi; do
    steps=20; [ $c = trembl ] && steps=3; [ $c = semi ] && steps=5
    timeout -k 10 400 python bench.py --config $c --steps $steps --warmup 3 > $OUT/$c.json 2> $OUT/$c.err || { tail -20 $OUT/$c.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$c.json')); print('$c', round(d['ms_per_step'],3), '%.4g' % d['value'], d.get('roofline',{}).get('frac'), d.get('count_only'), [(k['kernel'], round(k['ms_per_build'],2)) for k in d.get('kernels',[])][:7])"
  done
  AB_CONFIG=semi bash tools/ab_variants.sh r04c/ab base notag || exit 1
fi
echo ALLDONE
