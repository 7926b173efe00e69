# one-off GPU session script (changes per call)
set -o pipefail
O=gpurun_out/r06m1; mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT tests/test_gpu_parity.py tests/test_depth_gpu.py -k "multi_mass or giant or big_bins or isobaric or tag_coll or spikes or list_grids" > $O/t1.log 2>&1; rc=$?; tail -3 $O/t1.log; [ $rc -eq 0 ] || exit $rc
SB="python bench.py --config semi --steps 3 --warmup 3 --no-cpu-baseline --no-cold --queries 0"
for r in 1 2; do
  DBI_LIB_PATH=tools/exp/nomg.so timeout -k 10 400 $SB > $O/nomg$r.log 2>&1 || exit 1
  timeout -k 10 400 $SB > $O/cur$r.log 2>&1 || exit 1
done
python3 tools/ab_table.py $O nomg1 cur1 nomg2 cur2
DBI_LIB_PATH=tools/exp/pclock.so timeout -k 10 400 python tools/chunk_phase.py semi > $O/pclock_semi.log 2>&1 || exit 1
timeout -k 10 900 $PT tests/test_scale_gpu.py -k "semi_slice" > $O/t2.log 2>&1; rc=$?; tail -3 $O/t2.log; exit $rc
