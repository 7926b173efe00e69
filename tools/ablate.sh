#!/bin/bash
# temporary: time chunk_sort under DBI_ABLATE masks
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ablate
for a in 0 1 2 4 8 15; do
  DBI_ABLATE=$a timeout -k 10 120 python bench.py --steps 10 --warmup 2 --queries 0 --no-cpu-baseline > gpurun_out/ablate/a$a.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/ablate/a$a.json'))
k={x['kernel']:x['ms_per_build'] for x in d['kernels']}
print('ablate $a chunk_sort %.1f us  digest_count %.1f emit %.1f total %.1f'%(k['chunk_sort']*1e3, k['digest_count']*1e3, k['digest_emit']*1e3, d['ms_per_step']*1e3))"
done
