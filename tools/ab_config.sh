#!/bin/bash
# tools/ab_config.sh TAG CONFIG STEPS variant... — one config's build time for
# experiment builds (dbindex_amd/exp/<variant>.so; "base" = the in-tree build)
set -u -o pipefail
TAG=$1; C=$2; S=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
for v in "$@"; do
    if [ "$v" = base ]; then unset DBI_LIB_PATH; else export DBI_LIB_PATH=dbindex_amd/exp/$v.so; fi
    timeout -k 10 400 python bench.py --config $C --steps $S --warmup 2 --no-cpu-baseline --queries 0 > "$OUT/$v.json" 2> "$OUT/$v.err" \
        || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1])
print('$v', round(d['ms_per_step'],3), [(k['kernel'], round(k['ms_per_build'],3)) for k in d['kernels']][:7])"
done
