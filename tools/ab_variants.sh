#!/bin/bash
# tools/ab_variants.sh TAG variant... — bench experiment builds of the library
# (dbindex_amd/exp/<variant>.so via DBI_LIB_PATH; "base" = the in-tree build;
# AB_CONFIG=human etc. for another config; env-NAME=VALUE: the in-tree build
# with that environment variable)
set -u -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"
for spec in "$@"; do
    IFS=: read -r v ct <<< "$spec"   # variant[:chunk target]
    if [ -n "${ct:-}" ]; then export DBI_CHUNK_T=$ct; else unset DBI_CHUNK_T; fi
    envset=()
    if [ "${v#env-}" != "$v" ]; then  # env-NAME=VALUE: the in-tree build with that variable set
        envset=("${v#env-}"); unset DBI_LIB_PATH
    elif [ "$v" = base ]; then unset DBI_LIB_PATH; else export DBI_LIB_PATH=dbindex_amd/exp/$v.so; fi
    name=$v${ct:+_$ct}
    timeout -k 10 200 env "${envset[@]}" python bench.py --config "${AB_CONFIG:-swissprot}" --steps 10 --warmup 3 --no-cpu-baseline --queries 0 > "$OUT/$name.json" 2> "$OUT/$name.err" \
        || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],3), [(k['kernel'], round(k['ms_per_build'],3)) for k in d['kernels']][:6])"
done
