#!/bin/bash
# tools/ab_env.sh TAG CONFIG NAME=OPTIONS... — bench lines of the in-tree build
# under engine-option variants (e.g. "b16=bin_bits_max=16", "radix=depth_bins=0",
# "both=depth_bins=0,bin_bits_max=16", "base=") into gpurun_out/TAG/, one line
# of per-stage times each; stops at the first failure.
set -u -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for spec in "$@"; do
    name=${spec%%=*}; opts=${spec#*=}
    args=()
    IFS=, read -ra kv <<< "$opts"
    for o in "${kv[@]}"; do [ -n "$o" ] && args+=(--option "$o"); done
    timeout -k 10 300 python bench.py --config "$CFG" --steps ${AB_STEPS:-20} --warmup 5 --no-cpu-baseline --queries 0 --no-cold "${args[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err" \
        || { echo "$name failed"; tail -5 "$OUT/$name.err"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
print('$name', round(d['ms_per_step'],4), d['config'].get('n_bins'), [(k['kernel'], round(k['ms_per_build'],4)) for k in d['kernels']][:12])"
done
