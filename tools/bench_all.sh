#!/bin/bash
# tools/bench_all.sh TAG — every BASELINE config's bench line (one GPU) into
# gpurun_out/TAG/<config>.json; stops at the first failure.
set -u -o pipefail
TAG=${1:-bench}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for c in swissprot human semi trembl; do
  steps=20; [ $c = semi ] && steps=5; [ $c = trembl ] && steps=3
  timeout -k 10 600 python bench.py --config $c --steps $steps --warmup 5 > "$OUT/$c.json" 2> "$OUT/$c.err" || { tail -20 "$OUT/$c.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$c.json')); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'])"
done
timeout -k 10 600 python bench.py --merge --steps 20 --warmup 5 > "$OUT/swissprot_merge.json" 2> "$OUT/swissprot_merge.err" || { tail -20 "$OUT/swissprot_merge.err"; exit 1; }
echo ALLDONE
