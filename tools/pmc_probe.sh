#!/bin/bash
# tools/pmc_probe.sh TAG "COUNTERS..." — one rocprofv3 PMC pass over a short bench
set -u -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"; export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run \
     -- python3 bench.py --steps 3 --warmup 1 --queries 0 --no-cpu-baseline > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $set"
done
