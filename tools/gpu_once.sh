# one-off GPU session script (changes per call): tests then the e2e bench
set -o pipefail
mkdir -p gpurun_out/r06t6
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_fasta_gpu.py > gpurun_out/r06t6/t_fasta.log 2>&1 && tail -3 gpurun_out/r06t6/t_fasta.log && bash tools/gpu_r06.sh r06t6 e2e
