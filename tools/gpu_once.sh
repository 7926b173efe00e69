# one-off GPU session script (changes per call)
set -o pipefail
bash tools/gpu_r06.sh r06t9 t_all e2e
