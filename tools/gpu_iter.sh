#!/bin/bash
# tools/gpu_iter.sh TAG [tests|quick] — one build-iteration on the GPU box:
# parity tests (all, or the fast parity subset), the SwissProt bench line and
# a rocprofv3 kernel-trace + stats pass.  Stops at the first failure.
set -u -o pipefail
TAG=${1:-it}; MODE=${2:-quick}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$MODE" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scale_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "not semi_full" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
fi
tail -1 "$OUT/tests.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --queries 0 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
python3 tools/prof_summary.py "$OUT" "$OUT/summary" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
echo ALLDONE
