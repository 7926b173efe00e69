#!/bin/bash
# tools/ab_env.sh TAG CONFIG NAME=ENVSPEC... — bench lines of the in-tree build
# under environment variants (e.g. "b16=DBI_BIN_BITS_MAX=16", "base=") into
# gpurun_out/TAG/, one line of per-stage times each; stops at the first failure.
set -u -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    env $envs timeout -k 10 300 python bench.py --config "$CFG" --steps ${AB_STEPS:-20} --warmup 5 --no-cpu-baseline --queries 0 > "$OUT/$name.json" 2> "$OUT/$name.err" \
        || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],4), d['config'].get('n_bins'), [(k['kernel'], round(k['ms_per_build'],4)) for k in d['kernels']][:12])"
done
