#!/bin/bash
# tools/gpu_check.sh TAG [configs...] — the GPU test suite, then the named
# configs' bench lines (default: swissprot human semi) into gpurun_out/TAG/;
# stops at the first failure.
set -u -o pipefail
TAG=${1:-chk}; shift || true
CFGS=${*:-swissprot human semi}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1 || { tail -30 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
for c in $CFGS; do
  steps=20; [ $c = semi ] && steps=5; [ $c = trembl ] && steps=3
  timeout -k 10 600 python bench.py --config $c --steps $steps --warmup 5 > "$OUT/$c.json" 2> "$OUT/$c.err" || { tail -20 "$OUT/$c.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$c.json')); print('$c', round(d['ms_per_step'],3), '%.3g' % d['value'], [(k['kernel'], round(k['ms_per_build'],3)) for k in d['kernels']][:8])"
done
echo CHECK_DONE
