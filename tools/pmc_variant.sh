#!/bin/bash
# tools/pmc_variant.sh TAG VARIANT — SQ counters of one experiment build (or "base")
set -u -o pipefail
TAG=$1; V=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"; export TMPDIR=/tmp
if [ "$V" != base ]; then export DBI_LIB_PATH=dbindex_amd/exp/$V.so; fi
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    --output-format csv -d "$OUT/$V" -o run -- python3 bench.py --steps 3 --warmup 1 --queries 0 --no-cpu-baseline > "$OUT/$V.log" 2>&1
