#!/bin/bash
# tools/round_profile.sh TAG — the round's committed evidence in one GPU call:
# rocprofv3 kernel trace + stats and the FETCH/WRITE counter passes of the
# SwissProt build (gpu_round.sh prof pmc), their summary (also written into
# profiles/ on the box, so the bench lines read this round's traffic), the SQ
# counter pass, and every config's bench line (bench_all.sh).  Stops at the
# first failure.  Copy gpurun_out/TAG/summary_* to profiles/TAG_swissprot_*
# and gpurun_out/TAG/bench/*.json to profiles/TAG_*_bench.json afterwards.
set -u -o pipefail
TAG=${1:-r}
bash tools/gpu_round.sh "$TAG" prof pmc || exit 1
python3 tools/prof_summary.py "gpurun_out/$TAG" "gpurun_out/$TAG/summary" > "gpurun_out/$TAG/summary.txt" || exit 1
python3 tools/prof_summary.py "gpurun_out/$TAG" "profiles/${TAG}_swissprot" > /dev/null || exit 1
cat "gpurun_out/$TAG/summary.txt"
bash tools/gpu_round.sh "$TAG" pmc_sq || exit 1
python3 tools/sq_summary.py "gpurun_out/$TAG/pmc_sq" > "gpurun_out/$TAG/sq_summary.txt" || exit 1
bash tools/bench_all.sh "$TAG/bench" || exit 1
echo ROUND_PROFILE_DONE
