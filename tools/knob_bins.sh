#!/bin/bash
# semi-tryptic bench at several fine-bin counts
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/knob
for b in 24 25 26 27; do
  DBI_BIN_BITS_MAX=$b timeout -k 10 300 python bench.py --config semi --steps 4 --warmup 2 --no-cpu-baseline --queries 0 > gpurun_out/knob/b$b.json 2> gpurun_out/knob/b$b.err || { echo "b$b failed"; tail -5 gpurun_out/knob/b$b.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/knob/b$b.json'))
print('bits $b', round(d['ms_per_step'],1), d['config']['n_bins'], [(k['kernel'], round(k['ms_per_build'],1)) for k in d['kernels'][:8]])"
done
