# one-off GPU session script (changes per call): the bench's lean timed loop against the previous one
set -o pipefail
O=gpurun_out/r06l2; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu-baseline --no-cold --queries 0"
for r in 1 2 3; do
  timeout -k 10 300 python bench_prev_tmp.py $A > $O/prev$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $A > $O/cur$r.log 2>&1 || exit 1
done
python3 tools/ab_table.py $O prev1 cur1 prev2 cur2 prev3 cur3
timeout -k 10 300 python bench.py --config human $A > $O/human.log 2>&1 || exit 1
tail -c 300 $O/human.log
