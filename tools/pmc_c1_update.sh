#!/bin/bash
# PMC passes over the C1 step with the embedding update's passes as their own launches
# (--tbe-role 0), eager: bash tools/pmc_c1_update.sh <outdir>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/$1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"; do
  n=$(echo "$C" | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/$n" -o pmc \
    -- python3 "$ROOT/bench.py" --config small --tbe-role 0 --no-cpu-baseline --no-kernel-timing \
    --no-graph --preheat-ms 0 --steps 3 --warmup 2 > "$OUT/$n.json" 2> "$OUT/$n.err" || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "update_pass" in k or "tiled" in k or "presort" in k or "keys_hist" in k:
        print(k, {c: round(sum(v) / max(1, len(v)), 1) for c, v in d.items()})
PY
