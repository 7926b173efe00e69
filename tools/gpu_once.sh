# one-off GPU session script (changes per call): tests + A/B of the folded resets
set -o pipefail
O=gpurun_out/r06z2; mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 1000 $PT tests/test_depth_gpu.py tests/test_graph_gpu.py tests/test_gpu_parity.py tests/test_fasta_gpu.py tests/test_scale_gpu.py -k "not trembl" > $O/t1.log 2>&1; rc=$?; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
A="--steps 20 --warmup 5 --no-cpu-baseline --no-cold --queries 0"
for r in 1 2 3; do
  DBI_LIB_PATH=tools/exp/prev.so timeout -k 10 300 python bench.py $A > $O/prev$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $A > $O/cur$r.log 2>&1 || exit 1
done
python3 tools/ab_table.py $O prev1 cur1 prev2 cur2 prev3 cur3
for r in 1 2; do
  DBI_LIB_PATH=tools/exp/prev.so timeout -k 10 300 python bench.py --config human $A > $O/hprev$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --config human $A > $O/hcur$r.log 2>&1 || exit 1
done
python3 tools/ab_table.py $O hprev1 hcur1 hprev2 hcur2
