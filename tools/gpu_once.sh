# one-off GPU session script (changes per call): A/B of the depth chunk target with the big tier beside the chunk sort
set -o pipefail
O=gpurun_out/r06ct; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu-baseline --no-cold --queries 0"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/d$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $A --option chunk_target=1536 > $O/t1536_$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $A --option chunk_target=1664 > $O/t1664_$r.log 2>&1 || exit 1
done
python3 tools/ab_table.py $O d1 t1536_1 t1664_1 d2 t1536_2 t1664_2
