#!/bin/bash
# sort-path parity tests, then A/B bench lines: (mass rank, tag) counting sort on / off (semi, swissprot) and finalize block shapes
set -u -o pipefail
OUT=gpurun_out/${TAG:-r04w}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -k "giant or semi_slice or wide or collision or big_bins or isobaric or swissprot_full or grids" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 || { tail -60 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
AB_STEPS=8 bash tools/ab_env.sh $(basename $OUT)/semi semi mt1= mt0=DBI_MASS_TAG=0 || exit 1
bash tools/ab_env.sh $(basename $OUT)/sp swissprot mt1= mt0=DBI_MASS_TAG=0 f1=DBI_FIN=1 f2=DBI_FIN=2 f3=DBI_FIN=3 mt1b= f1b=DBI_FIN=1 || exit 1
echo ALLDONE
