#!/bin/bash
# Kernel-trace timeline of one replayed bench step:  bash tools/step_trace.sh <outdir> [bench args]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/$1
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o kt \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-timing --steps 30 --warmup 10 "$@" \
  > "$OUT/b.json" 2> "$OUT/b.err" || exit $?
f=$(find "$OUT/kt" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/tools/step_timeline.py" "$f" > "$OUT/timeline.txt" || exit $?
cat "$OUT/timeline.txt"
