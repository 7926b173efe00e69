#!/bin/bash
# finalize block shape: the GPU suite, then A/B bench lines (512 x 4 default vs 256 x 4) on every materialised config
set -u -o pipefail
OUT=gpurun_out/${TAG:-r04x}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
bash tools/ab_env.sh $(basename $OUT)/human human f512= f256=DBI_FIN=1 f512b= f256b=DBI_FIN=1 || exit 1
AB_STEPS=8 bash tools/ab_env.sh $(basename $OUT)/semi semi f512= f256=DBI_FIN=1 || exit 1
bash tools/ab_env.sh $(basename $OUT)/sp swissprot f512= f256=DBI_FIN=1 f512b= f256b=DBI_FIN=1 || exit 1
echo ALLDONE
