# one-off GPU session script (changes per call)
set -o pipefail
mkdir -p gpurun_out/r06t8
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_fasta_gpu.py -k "fused" > gpurun_out/r06t8/t_fasta.log 2>&1 && tail -3 gpurun_out/r06t8/t_fasta.log && bash tools/gpu_r06.sh r06t8 e2e e2e_trace_fasta
