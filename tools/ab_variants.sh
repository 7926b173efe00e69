#!/bin/bash
# tools/ab_variants.sh TAG variant... — bench experiment builds of the library
# (dbindex_amd/exp/<variant>.so via DBI_LIB_PATH; "base" = the in-tree build;
# AB_CONFIG=human etc. for another config; variant:NAME=VALUE adds the engine
# option NAME=VALUE, e.g. base:chunk_target=3072)
set -u -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
for spec in "$@"; do
    IFS=: read -r v opt <<< "$spec"   # variant[:option]
    args=()
    if [ -n "${opt:-}" ]; then args=(--option "$opt"); fi
    if [ "$v" = base ]; then unset DBI_LIB_PATH; else export DBI_LIB_PATH=dbindex_amd/exp/$v.so; fi
    name=$v${opt:+_${opt//=/}}
    timeout -k 10 200 python bench.py --config "${AB_CONFIG:-swissprot}" --steps 10 --warmup 5 --no-cpu-baseline --queries 0 --no-cold "${args[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err" \
        || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],3), [(k['kernel'], round(k['ms_per_build'],3)) for k in d['kernels']][:6])"
done
