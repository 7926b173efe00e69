#!/bin/bash
# tools/gpu_round.sh TAG [what...] — one GPU-box session: parity tests, bench,
# rocprofv3 kernel trace + stats, HBM counter passes.  Every GPU step has its
# own time limit; the script stops at the first failure.
#   what: tests smoke bench bench_h prof prof_semi pmc pmc_sq pmc_sq_trembl (default: tests bench prof)
set -u -o pipefail
TAG=${1:-r}
shift || true
WHAT=${*:-tests bench prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
step() {  # name timeout cmd...
    local name=$1 to=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name exit $rc"
    tail -5 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
for w in $WHAT; do
    case $w in
    tests) step tests 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --steps 20 --warmup 5
           cp "$OUT/bench.log" "$OUT/bench.json" ;;
    bench_h) step bench_h 600 python bench.py --config human --steps 20 --warmup 5 ;;
    prof)  export TMPDIR=/tmp
           step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
                -- python3 bench.py --steps 10 --warmup 3 --queries 0 --no-cpu-baseline --no-cold ;;
    prof_semi) export TMPDIR=/tmp
           step prof_semi 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_semi" -o run \
                -- python3 bench.py --config semi --steps 4 --warmup 5 --queries 0 --no-cpu-baseline --no-cold ;;
    pmc)   export TMPDIR=/tmp
           step pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
                -- python3 bench.py --steps 5 --warmup 3 --queries 0 --no-cpu-baseline --no-cold
           step pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
                -- python3 bench.py --steps 5 --warmup 3 --queries 0 --no-cpu-baseline --no-cold ;;
    pmc_semi) export TMPDIR=/tmp
           step pmc_semi_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/semi/pmc_fetch" -o run \
                -- python3 bench.py --config semi --steps 2 --warmup 3 --queries 0 --no-cpu-baseline --no-cold
           step pmc_semi_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/semi/pmc_write" -o run \
                -- python3 bench.py --config semi --steps 2 --warmup 3 --queries 0 --no-cpu-baseline --no-cold
           step prof_semi2 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/semi/prof" -o run \
                -- python3 bench.py --config semi --steps 2 --warmup 3 --queries 0 --no-cpu-baseline --no-cold ;;
    pmc_sq_trembl) export TMPDIR=/tmp
           step pmc_sq_trembl 900 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
                --output-format csv -d "$OUT/trembl_sq" -o run \
                -- python3 bench.py --config trembl --steps 1 --warmup 0 --no-cpu-baseline ;;
    pmc_sq) export TMPDIR=/tmp
           step pmc_sq 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
                --output-format csv -d "$OUT/pmc_sq" -o run \
                -- python3 bench.py --steps 5 --warmup 3 --queries 0 --no-cpu-baseline --no-cold ;;
    esac
done
echo ALLDONE
