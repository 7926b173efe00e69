# one-off GPU session script (changes per call): TrEMBL bucket-count A/B of hist_advance's lookahead
set -o pipefail
O=gpurun_out/r06tl; mkdir -p $O
A="--config trembl --trembl-proteins 10000000 --steps 4 --warmup 1 --no-cold --queries 0"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/cur$r.log 2>&1 || exit 1
  DBI_LIB_PATH=tools/exp/look2.so timeout -k 10 300 python bench.py $A > $O/look2_$r.log 2>&1 || exit 1
done
for f in $O/*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2), d["cpu_baseline"].get("sample_bucket_parity"))')"; done
