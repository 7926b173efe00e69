#!/bin/bash
# tools/gpu_r06.sh TAG STEP... — one GPU-box session of round 6.  Every GPU step
# has its own time limit; the script stops at the first failure.
#   t_depth   tests/test_depth_gpu.py
#   t_scale   the SwissProt-scale parity tests (full tryptic + 8 shards)
#   t_all     the whole GPU suite
#   ab_stage  bench SwissProt with part_stage=1, 0, 1 (A/B on one box)
#   bench     the driver's bench line (default flags)
#   prof      rocprofv3 kernel trace + stats of the bench (SwissProt)
#   pmc       FETCH_SIZE / WRITE_SIZE passes (SwissProt)
#   sq        SQ counter pass (SwissProt)
#   semi      semi bench, semi trace + PMC
#   h2d       tools/probe/h2d_probe (host-to-device copy paths)
#   ring      tools/probe/h2d_ring (the residue upload's staged-ring variants)
#   dclock    digest phase clocks (tools/exp/dclock.so)
#   sq_trembl SQ counter pass of the TrEMBL bench (the bucket kernel's VALU count)
#   pclock    chunk-sort phase clocks, semi and SwissProt (tools/exp/pclock.so)
#   noverify  chunk-sort traffic with / without string verification (tools/exp/noverify.so)
#   ab_prev   bench of tools/exp/prev.so (the last commit) against the tree, twice each
#   allconf   tools/bench_all.sh: every config's bench line (+ --merge)
#   budget    tools/shard_budget.py (N = 8 model, 12 builds)
#   e2e       bench with the cold / end-to-end legs, no CPU baseline
#   e2e_trace HIP API + kernel + copy trace of fresh engines' builds (tools/e2e_trace.py)
set -u -o pipefail
TAG=${1:-r06}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
    local name=$1 to=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name exit $rc"
    tail -4 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold --queries 0"
for w in "$@"; do
    case $w in
    t_depth) step t_depth 600 $PT tests/test_depth_gpu.py ;;
    t_graph) step t_graph 600 $PT tests/test_graph_gpu.py tests/test_depth_gpu.py ;;
    t_scale) step t_scale 900 $PT tests/test_scale_gpu.py -k "full_tryptic or sharded_8 or semi_slice" ;;
    t_all)   step t_all 1100 $PT tests -m gpu ;;
    ab_stage) step ab1 300 $B --option part_stage=1
              step ab0 300 $B --option part_stage=0
              step ab1b 300 $B --option part_stage=1 ;;
    bench)   step bench 600 python bench.py --steps 20 --warmup 5 ;;
    bench_h) step bench_h 300 python bench.py --config human --steps 20 --warmup 5 --no-cpu-baseline ;;
    prof)    step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run \
                -- python3 bench.py --steps 10 --warmup 5 --queries 0 --no-cpu-baseline --no-cold ;;
    pmc)     step pmc_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
                -- python3 bench.py --steps 5 --warmup 5 --queries 0 --no-cpu-baseline --no-cold
             step pmc_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
                -- python3 bench.py --steps 5 --warmup 5 --queries 0 --no-cpu-baseline --no-cold ;;
    sq)      step pmc_sq 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
                --output-format csv -d "$OUT/pmc_sq" -o run \
                -- python3 bench.py --steps 5 --warmup 5 --queries 0 --no-cpu-baseline --no-cold ;;
    semi)    step semi_bench 600 python bench.py --config semi --steps 5 --warmup 5 --no-cpu-baseline --no-cold --queries 0
             step semi_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/semi/prof" -o run \
                -- python3 bench.py --config semi --steps 2 --warmup 4 --queries 0 --no-cpu-baseline --no-cold ;;
    semi_pmc) step semi_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/semi/pmc_fetch" -o run \
                -- python3 bench.py --config semi --steps 2 --warmup 4 --queries 0 --no-cpu-baseline --no-cold
             step semi_write 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/semi/pmc_write" -o run \
                -- python3 bench.py --config semi --steps 2 --warmup 4 --queries 0 --no-cpu-baseline --no-cold ;;
    h2d)     step h2d 180 ./tools/probe/h2d_probe ;;
    ring)    step ring 240 ./tools/probe/h2d_ring ;;
    dclock)  export DBI_LIB_PATH=tools/exp/dclock.so
             step dclock 300 python tools/digest_phase.py
             unset DBI_LIB_PATH ;;
    noverify) step noverify 900 bash tools/exp_pmc.sh $TAG/exp base noverify ;;
    ab_prev) for r in 1 2; do
                 DBI_LIB_PATH=tools/exp/prev.so step prev$r 300 $B
                 step cur$r 300 $B
             done
             python3 tools/ab_table.py "$OUT" prev1 cur1 prev2 cur2 ;;
    ab3)     for r in 1 2; do   # ab3 A B: tools/exp/A.so, tools/exp/B.so and the tree
                 DBI_LIB_PATH=tools/exp/$V1.so step ${V1}$r 300 $B
                 DBI_LIB_PATH=tools/exp/$V2.so step ${V2}$r 300 $B
                 step cur$r 300 $B
             done
             python3 tools/ab_table.py "$OUT" ${V1}1 ${V2}1 cur1 ${V1}2 ${V2}2 cur2 ;;
    allconf) step allconf 1100 bash tools/bench_all.sh $TAG/bench ;;
    budget)  step budget 900 bash -c "python tools/shard_budget.py --reps 12 > $OUT/shard_budget8.json" ;;
    e2e)     step e2e 300 python bench.py --steps 10 --warmup 5 --no-cpu-baseline --queries 0 ;;
    e2e_trace) step e2e_trace 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv \
                -d "$OUT/trace" -o run -- python3 tools/e2e_trace.py
             python3 tools/api_timeline.py "$OUT/trace" > "$OUT/e2e_timeline.txt" ;;
    e2e_trace_fasta) step e2e_trace_fasta 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv \
                -d "$OUT/trace_fasta" -o run -- python3 tools/e2e_trace.py swissprot fasta
             python3 tools/api_timeline.py "$OUT/trace_fasta" > "$OUT/e2e_fasta_timeline.txt" ;;
    pclock)  export DBI_LIB_PATH=tools/exp/pclock.so
             step pclock_semi 400 python tools/chunk_phase.py semi
             step pclock_sp 300 python tools/chunk_phase.py swissprot
             unset DBI_LIB_PATH ;;
    sq_trembl) step pmc_sq_trembl 900 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
                --output-format csv -d "$OUT/trembl_sq" -o run \
                -- python3 bench.py --config trembl --steps 1 --warmup 0 --no-cpu-baseline
             python3 tools/sq_kernel_totals.py "$OUT/trembl_sq" > "$OUT/trembl_sq.json" ;;
    *) echo "unknown step $w"; exit 2 ;;
    esac
done
echo ALLDONE
