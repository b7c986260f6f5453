#!/bin/bash
# Alternating A/B of two DLRM_WG_SPLITS settings ($1 vs $2), N rounds, full C3 step.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/wgab
mkdir -p "$OUT"
for r in ${ROUNDS:-1 2 3 4}; do
  for cfg in "$1" "$2"; do
    DLRM_WG_SPLITS="$cfg" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 500 \
      > "$OUT/b.json" 2> "$OUT/b.err" || exit 1
    python -c "import json; d=json.load(open('$OUT/b.json')); print(repr('$cfg'), d['value'], d['kernel_us_per_step']['gemm'])"
  done
done
