#!/bin/bash
# Interleaved A/B of one bench flag's values in one GPU session:
#   bash tools/ab_flag.sh <outdir> <rounds> "<flag>" "<v1 v2 ...>" [bench args]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/$1; N=$2; FLAG=$3; VALS=$4; shift 4
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  for v in $VALS; do
    timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-timing --steps 300 \
      --warmup 30 $FLAG "$v" "$@" > "$OUT/$v.$i.json" 2> "$OUT/$v.$i.err" || exit $?
    python3 -c "import json,sys; d=json.load(open('$OUT/$v.$i.json')); print('$FLAG $v', d['value'], d['ms_per_step'], d['ms_per_step_p10_p50_p90'])" | tee -a "$OUT/ab.txt"
  done
done
