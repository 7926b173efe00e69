#!/bin/bash
# A/B: bench with per-kernel dispatch-packet events on vs wall clock only
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/ab
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --queries 0 --no-cpu-baseline --timing off > gpurun_out/ab/off.json 2> gpurun_out/ab/off.err || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --queries 0 --no-cpu-baseline --timing on > gpurun_out/ab/on.json 2> gpurun_out/ab/on.err || exit 1
python3 -c "
import json
for t in ('on','off'):
    d=json.load(open('gpurun_out/ab/%s.json'%t)); print(t, d['ms_per_step'], d['value'], sum(k['ms_per_build'] for k in d['kernels']))
"
