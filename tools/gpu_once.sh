# one-off GPU session script (changes per call): tests + A/B of the side big tier (two size classes) against in line
set -o pipefail
O=gpurun_out/r06bs5; mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_depth_gpu.py tests/test_graph_gpu.py tests/test_scale_gpu.py tests/test_gpu_parity.py -k "not trembl and not semi" > $O/t1.log 2>&1; rc=$?; tail -2 $O/t1.log; [ $rc -eq 0 ] || exit $rc
A="--steps 20 --warmup 5 --no-cpu-baseline --no-cold --queries 0"
for r in 1 2 3; do
  timeout -k 10 300 python bench.py $A --option big_side=0 > $O/off$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $A > $O/on$r.log 2>&1 || exit 1
done
python3 tools/ab_table.py $O off1 on1 off2 on2 off3 on3
