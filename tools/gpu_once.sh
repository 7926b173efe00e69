# one-off GPU session script (changes per call): depth / graph tests + A/B of the big tier beside the chunk sort
set -o pipefail
O=gpurun_out/r06bs4; mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_depth_gpu.py tests/test_graph_gpu.py tests/test_scale_gpu.py tests/test_shard_gpu.py -k "not trembl and not semi" > $O/t1.log 2>&1; rc=$?; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
A="--steps 20 --warmup 5 --no-cpu-baseline --no-cold --queries 0"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A --option big_side=0 > $O/off$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $A > $O/on$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --config human $A --option big_side=0 > $O/hoff$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --config human $A > $O/hon$r.log 2>&1 || exit 1
done
python3 tools/ab_table.py $O off1 on1 off2 on2 hoff1 hon1 hoff2 hon2
