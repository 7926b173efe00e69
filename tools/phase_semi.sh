#!/bin/bash
# per-phase clocks of the chunk-sort kernels (DBI_X_PHASE build) on a config
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/phase
C=${1:-semi}
DBI_LIB_PATH=dbindex_amd/exp/phase.so timeout -k 10 300 python bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --queries 0 > gpurun_out/phase/$C.json 2> gpurun_out/phase/$C.err || { tail -5 gpurun_out/phase/$C.err; exit 1; }
grep "^phase" gpurun_out/phase/$C.err | tail -3
