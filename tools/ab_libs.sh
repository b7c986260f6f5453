#!/bin/bash
# Interleaved A/B of two builds of libdlrm_hip.so in one GPU session:
#   bash tools/ab_libs.sh <outdir> <rounds> [bench args]   (${ABDIR:-tools/_ab}/libA.so, tools/_ab/libB.so)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/$1; N=$2; shift 2
mkdir -p "$OUT"
LIB=$ROOT/dlrm-yx_amd/dlrm_hip/libdlrm_hip.so
for i in $(seq 1 "$N"); do
  for v in ${VARIANTS:-A B}; do
    cp "$ROOT/${ABDIR:-tools/_ab}/lib$v.so" "$LIB" || exit 1
    timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-timing --steps 300 \
      --warmup 30 "$@" > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || exit $?
    python3 -c "import json,sys; d=json.load(open('$OUT/$v$i.json')); print('$v', d['value'], d['ms_per_step'], d['ms_per_step_p10_p50_p90'])" | tee -a "$OUT/ab.txt"
  done
done
