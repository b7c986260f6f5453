#!/bin/bash
# One GPU session: parity tests, the bench line, a rocprofv3 kernel-trace summary of the
# same bench command and two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic.
# Usage (from the repo root, on the GPU box):  bash tools/gpu_round.sh [tag] [stages]
#   stages: any of t (tests) b (bench) p (profile) c (counters); default "tbpc"
set -o pipefail
TAG=${1:-r01}
STAGES=${2:-tbpc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT" || exit 1
if [[ $STAGES == *t* ]]; then
  echo "[gpu_round] pytest -m gpu"
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STAGES == *b* ]]; then
  echo "[gpu_round] bench"
  timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
  cat "$OUT/bench.json"
fi
BENCH_ARGS="--no-cpu-baseline --steps 50 --warmup 10"
cd /tmp && export TMPDIR=/tmp
if [[ $STAGES == *p* ]]; then
  echo "[gpu_round] rocprofv3 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" \
    -o kt -- python3 "$ROOT/bench.py" $BENCH_ARGS > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || exit $?
fi
if [[ $STAGES == *c* ]]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "[gpu_round] rocprofv3 --pmc $C"
    timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-timing --no-graph --steps 10 \
      --warmup 2 > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err" || exit $?
  done
fi
echo "[gpu_round] done"
