#!/bin/bash
# tools/ab_queries_cfg.sh TAG CONFIG variant... — query legs of one config for experiment builds
set -u -o pipefail
TAG=$1; C=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
for v in "$@"; do
    if [ "$v" = base ]; then unset DBI_LIB_PATH; else export DBI_LIB_PATH=dbindex_amd/exp/$v.so; fi
    timeout -k 10 400 python bench.py --config $C --steps 2 --warmup 2 --no-cpu-baseline > "$OUT/$C-$v.json" 2> "$OUT/$C-$v.err" \
        || { echo "$v failed"; tail -5 "$OUT/$C-$v.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/$C-$v.json').read().strip().splitlines()[-1]); q=d['queries']; m=q['materialised']
print('$C $v', 'range %.3g q/s' % q['value'], 'materialised %.3g q/s %.2f ms/batch frac %.3f' % (m['value'], m['ms_per_batch'], m['roofline']['frac']))"
done
