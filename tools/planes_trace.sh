#!/bin/bash
# Kernel trace of the C3 step with the top MLP on split-bf16 planes (DLRM_GEMM_PLANES=1) and
# on the exact-f32 body (=0): per-launch timeline of one replayed step each.
#   bash tools/planes_trace.sh <outdir>
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/${1:-gpurun_out/planes}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for pl in 1 0; do
  DLRM_GEMM_PLANES=$pl timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
    -d "$OUT/kt$pl" -o kt -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-timing \
    --steps 30 --warmup 10 > "$OUT/b$pl.json" 2> "$OUT/b$pl.err" || exit $?
  f=$(find "$OUT/kt$pl" -name "*kernel_trace.csv" | head -1)
  python3 "$ROOT/tools/step_timeline.py" "$f" > "$OUT/timeline$pl.txt" || exit $?
  echo "== planes=$pl"; cat "$OUT/timeline$pl.txt"
done
