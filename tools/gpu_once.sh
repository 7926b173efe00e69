# one-off GPU session script (changes per call)
set -o pipefail
O=gpurun_out/r06k1; mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_parity.py tests/test_scale_gpu.py -k "count_buckets or trembl" > $O/t1.log 2>&1; rc=$?; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
TB="python bench.py --config trembl --trembl-proteins 10000000 --steps 5 --warmup 2 --no-cpu-baseline"
for r in 1 2; do
  DBI_LIB_PATH=tools/exp/prevkt.so timeout -k 10 400 $TB > $O/prev$r.log 2>&1 || exit 1
  timeout -k 10 400 $TB > $O/cur$r.log 2>&1 || exit 1
done
for f in prev1 cur1 prev2 cur2; do python3 -c "
import json,sys; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],2), 'count_only', round(d['count_only']['ms'],2), d['bucket_counts']['counts'][:3])"; done
