#!/bin/bash
# round-4 checkpoint on the restored tree: GPU suite, the round's profile set
# (rocprof stats + PMC + SQ + every config's bench line) and the 8-shard budget
set -u -o pipefail
TAG=${1:-r04e}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=3 -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
bash tools/round_profile.sh $TAG || exit 1
timeout -k 10 300 python tools/shard_budget.py --reps 4 > $OUT/budget.json 2> $OUT/budget.err || { tail -20 $OUT/budget.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/budget.json')); print('budget', d['front_ms'], d['exchange_model_ms'], d['merge_max_ms'], d.get('fixed_ms'), d.get('model_ms'))"
echo ALLDONE
