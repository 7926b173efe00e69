#!/bin/bash
# tools/exp_pmc.sh TAG variant... — FETCH_SIZE / WRITE_SIZE passes of the SwissProt
# bench for experiment builds (tools/exp/<variant>.so; "base" = in-tree),
# with each kernel's traffic per launch (2 x FETCH + WRITE, MI355X_MICROARCH.md).
set -u -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"; cd "$ROOT"; export TMPDIR=/tmp
for v in "$@"; do
    if [ "$v" = base ]; then unset DBI_LIB_PATH; else export DBI_LIB_PATH=tools/exp/$v.so; fi
    timeout -k 10 200 python bench.py --steps 10 --warmup 5 --no-cpu-baseline --queries 0 --no-cold > "$OUT/$v.json" 2> "$OUT/$v.err" || { tail -5 "$OUT/$v.err"; exit 1; }
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/${v}_$c" -o run \
            -- python3 bench.py --steps 3 --warmup 3 --queries 0 --no-cpu-baseline --no-cold > "$OUT/${v}_$c.log" 2>&1 || { tail -5 "$OUT/${v}_$c.log"; exit 1; }
    done
    python3 - "$OUT" "$v" <<'PY'
import csv, glob, json, sys, collections
out, v = sys.argv[1], sys.argv[2]
d = json.loads(open(f"{out}/{v}.json").read().strip().splitlines()[-1])
tot = collections.defaultdict(lambda: [0.0, 0])
for c, mul in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
    f = glob.glob(f"{out}/{v}_{c}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, vals in per.items():
        vals = sorted(vals)[len(vals) // 4:]  # the later (steady) launches dominate
        tot[k][0] += mul * sum(vals) / len(vals) * 1024 / 1e6  # KB -> MB per launch
        tot[k][1] = max(tot[k][1], len(vals))
print(v, "ms/build", round(d["ms_per_step"], 3))
for k, (mb, n) in sorted(tot.items(), key=lambda x: -x[1][0])[:8]:
    print(f"   {k[:60]:60s} {mb:9.1f} MB/launch")
PY
done
echo ALLDONE
