#!/bin/bash
# tools/ab_semi.sh TAG variant... — semi-tryptic (configs[3]) bench of experiment
# builds (dbindex_amd/exp/<variant>.so; "base" = the in-tree build)
set -u -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for v in "$@"; do
    if [ "$v" = base ]; then unset DBI_LIB_PATH; else export DBI_LIB_PATH=dbindex_amd/exp/$v.so; fi
    timeout -k 10 300 python bench.py --config semi --steps 3 --warmup 2 --no-cpu-baseline --queries 0 > "$OUT/semi_$v.json" 2> "$OUT/semi_$v.err" \
        || { echo "$v failed"; tail -5 "$OUT/semi_$v.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/semi_$v.json').read().strip().splitlines()[-1])
print('semi $v', round(d['ms_per_step'],2), [(k['kernel'], round(k['ms_per_build'],2)) for k in d['kernels']][:7])"
done
