#!/bin/bash
# chunk sizes routed through the giant split (DBI_SPLIT_ABOVE) on swissprot and semi
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ksplit
for c in swissprot semi; do
  for v in 7936 1984; do
    st=8; [ $c = semi ] && st=3
    DBI_SPLIT_ABOVE=$v timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline --queries 0 > gpurun_out/ksplit/$c$v.json 2> gpurun_out/ksplit/$c$v.err || { echo "$c $v failed"; tail -5 gpurun_out/ksplit/$c$v.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/ksplit/$c$v.json'))
print('$c split>$v', round(d['ms_per_step'],2), [(k['kernel'], round(k['ms_per_build'],2)) for k in d['kernels'] if k['kernel'].startswith('chunk')])"
  done
done
