# one-off GPU session script (changes per call): the round-end steps
set -o pipefail
O=gpurun_out/r06f2; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > $O/t_all.log 2>&1; rc=$?; tail -3 $O/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; tail -c 600 $O/bench.json; exit $rc
