#!/bin/bash
# Sweep the K split of each top-MLP wgrad in the full C3 step (DLRM_WG_SPLITS), one bench
# run per setting; prints the GEMM group time per step and the step rate.
set -o pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/wgsweep
mkdir -p "$OUT"
run() {
  DLRM_WG_SPLITS="$1" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 \
    > "$OUT/b.json" 2> "$OUT/b.err" || exit 1
  python -c "import json; d=json.load(open('$OUT/b.json')); print('$1', d['value'], d['kernel_us_per_step']['gemm'])"
}
run ""
for L in ${LAYERS:-top0 top1 top2 top3}; do
  for s in 1 2 4 8; do run "$L:$s"; done
done
