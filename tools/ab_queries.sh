#!/bin/bash
# tools/ab_queries.sh TAG variant... — the query legs of experiment builds
# (dbindex_amd/exp/<variant>.so via DBI_LIB_PATH; "base" = the in-tree build)
set -u -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
for v in "$@"; do
    if [ "$v" = base ]; then unset DBI_LIB_PATH; else export DBI_LIB_PATH=dbindex_amd/exp/$v.so; fi
    timeout -k 10 200 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/$v.json" 2> "$OUT/$v.err" \
        || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); q=d['queries']; m=q['materialised']
print('$v', 'range %.3g q/s' % q['value'], 'materialised %.3g q/s %.2f ms/batch frac %.3f' % (m['value'], m['ms_per_batch'], m['roofline']['frac']))"
done
