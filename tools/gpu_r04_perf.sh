#!/bin/bash
# Round-4 perf session (one gpurun call):  bash tools/gpu_r04_perf.sh <stage>
#   ab      - C3 / C2 / C3@B=256 bench lines, bottom-backward schedule partial vs chain
#   trace   - one-step kernel timelines (C3 default, C2 default)
#   sweep   - GEMM plan sweeps: Kaggle shapes at B=128 and C3 shapes at B=256 (fwd splits)
set -o pipefail
STAGE=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${OUTNAME:-r04_perf}
mkdir -p "$OUT"
cd "$ROOT" || exit 1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing"
case $STAGE in
ab)
  for cfg in terabyte kaggle; do
    for s in partial chain; do
      $B --config $cfg --bot-sched $s --steps 300 --warmup 30 > "$OUT/ab_${cfg}_$s.json" \
        2> "$OUT/ab_${cfg}_$s.err" || exit $?
      python -c "import json,sys;d=json.load(open('$OUT/ab_${cfg}_$s.json'));print('$cfg $s',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
    done
  done
  for s in partial chain; do
    $B --batch 256 --bot-sched $s --steps 300 --warmup 30 > "$OUT/ab_b256_$s.json" \
      2> "$OUT/ab_b256_$s.err" || exit $?
    python -c "import json;d=json.load(open('$OUT/ab_b256_$s.json'));print('b256 $s',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
  done
  ;;
trace)
  bash tools/step_trace.sh gpurun_out/${OUTNAME:-r04_perf}/trace_c3 ${BOT:+--bot-sched $BOT} || exit $?
  bash tools/step_trace.sh gpurun_out/${OUTNAME:-r04_perf}/trace_c2 --config kaggle ${BOT:+--bot-sched $BOT} || exit $?
  ;;
sweep)
  timeout -k 10 500 python tools/gemm_sweep.py --batches 128 --layers kaggle --fwd-splits \
    --out "$OUT/plans_kaggle.json" > "$OUT/sweep_kaggle.txt" 2>&1 || exit $?
  tail -3 "$OUT/sweep_kaggle.txt"
  timeout -k 10 500 python tools/gemm_sweep.py --batches 256 --fwd-splits \
    --out "$OUT/plans_b256.json" > "$OUT/sweep_b256.txt" 2>&1 || exit $?
  tail -3 "$OUT/sweep_b256.txt"
  ;;
esac
