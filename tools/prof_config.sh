#!/bin/bash
# rocprofv3 kernel stats of one config's bench (tools/prof_config.sh TAG CONFIG)
set -u -o pipefail
TAG=$1; C=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
    -- python3 bench.py --config $C --steps 3 --warmup 1 --queries 0 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:16]: print(r['Name'][:90], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2), 'ms')
"
