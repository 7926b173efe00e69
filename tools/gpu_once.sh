# one-off GPU session script (changes per call): A/B of an experiment library
set -o pipefail
O=gpurun_out/r06o2; mkdir -p $O
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-cold --queries 0"
for r in 1 2 3; do
  DBI_LIB_PATH=tools/exp/optim.so timeout -k 10 300 $B > $O/optim$r.log 2>&1 || exit 1
  timeout -k 10 300 $B > $O/cur$r.log 2>&1 || exit 1
done
python3 tools/ab_table.py $O optim1 cur1 optim2 cur2 optim3 cur3
