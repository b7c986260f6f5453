#!/bin/bash
# Interleaved A/B of bench argument sets in one GPU session:
#   bash tools/ab_args.sh <outdir> <rounds> "<args A>" "<args B>" ...   (common args: $AB_COMMON)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/$1; N=$2; shift 2
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  v=0
  for a in "$@"; do
    v=$((v + 1))
    timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-timing --steps 300 \
      --warmup 30 $AB_COMMON $a > "$OUT/v$v.$i.json" 2> "$OUT/v$v.$i.err" || exit $?
    python3 -c "import json,sys; d=json.load(open('$OUT/v$v.$i.json')); print('[$a]', d['value'], d['ms_per_step'], d['ms_per_step_p10_p50_p90'])" | tee -a "$OUT/ab.txt"
  done
done
