#!/bin/bash
# tools/ab_knobs.sh TAG — bench the build under engine tuning knobs
# (DBI_BIN_BITS_MAX, DBI_SPLIT_ABOVE); one JSON summary line per setting.
set -u -o pipefail
TAG=${1:-ab}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
run() {  # name config env...
    local name=$1 cfg=$2; shift 2
    env "$@" timeout -k 10 300 python bench.py --config "$cfg" --steps 5 --warmup 2 --queries 0 --no-cpu-baseline \
        > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
k={x['kernel']:round(x['ms_per_build'],2) for x in d['kernels']}
print('$name', round(d['ms_per_step'],3), k)"
}
for spec in "$@"; do
    IFS=: read -r name cfg bits split ct <<< "$spec"
    run "$name" "$cfg" DBI_BIN_BITS_MAX=$bits DBI_SPLIT_ABOVE=$split DBI_CHUNK_T=${ct:-1024}
done
