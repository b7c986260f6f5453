#!/bin/bash
# Round-4 perf session (one gpurun call):  bash tools/gpu_r04_perf.sh <stage>
#   ab      - C3 / C2 / C3@B=256 bench lines, bottom-backward schedule partial vs chain
#   ab2     - CFGS x SCHEDS bottom-backward schedule A/B
#   role    - CFGS: the embedding update as GEMM-launch roles (--tbe-role 1) vs own launches
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
ab2)  # CFGS="terabyte kaggle b256" SCHEDS="partial full"
  for cfg in ${CFGS:-terabyte kaggle b256}; do
    for s in ${SCHEDS:-partial full}; do
      if [ "$cfg" = b256 ]; then a="--batch 256"; else a="--config $cfg"; fi
      $B $a --bot-sched $s --steps 300 --warmup 30 > "$OUT/ab_${cfg}_$s.json" \
        2> "$OUT/ab_${cfg}_$s.err" || exit $?
      python -c "import json;d=json.load(open('$OUT/ab_${cfg}_$s.json'));print('$cfg $s',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
    done
  done
  ;;
role)  # the embedding update as GEMM-launch roles vs own launches
  for cfg in ${CFGS:-terabyte kaggle b256}; do
    for r in 0 1; do
      if [ "$cfg" = b256 ]; then a="--batch 256"; else a="--config $cfg"; fi
      $B $a --tbe-role $r --steps 300 --warmup 30 > "$OUT/role_${cfg}_$r.json" \
        2> "$OUT/role_${cfg}_$r.err" || exit $?
      python -c "import json;d=json.load(open('$OUT/role_${cfg}_$r.json'));print('$cfg role=$r',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
    done
  done
  ;;
roleat)  # placement of the two passes: AT="0,1 0,2 ..."
  for cfg in ${CFGS:-terabyte kaggle b256}; do
    for at in ${AT:-0,1 0,2 0,3 1,2}; do
      if [ "$cfg" = b256 ]; then a="--batch 256"; else a="--config $cfg"; fi
      $B $a --tbe-role-at $at --steps 300 --warmup 30 > "$OUT/at_${cfg}_$at.json" \
        2> "$OUT/at_${cfg}_$at.err" || exit $?
      python -c "import json;d=json.load(open('$OUT/at_${cfg}_$at.json'));print('$cfg at=$at',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
    done
  done
  ;;
parts)  # fused bottom MLP: one workgroup per 16-row block vs the auto split
  for cfg in ${CFGS:-kaggle b256}; do
    for pp in 1 0; do
      if [ "$cfg" = b256 ]; then a="--batch 256"; else a="--config $cfg"; fi
      $B $a --bottom-parts $pp --steps 300 --warmup 30 > "$OUT/parts_${cfg}_$pp.json" \
        2> "$OUT/parts_${cfg}_$pp.err" || exit $?
      python -c "import json;d=json.load(open('$OUT/parts_${cfg}_$pp.json'));print('$cfg parts=$pp',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
    done
  done
  ;;
sortab)  # the per-table sort: lookup launch vs a top-MLP forward launch (VARIANTS)
  for cfg in ${CFGS:-terabyte kaggle b256}; do
    for v in ${VARIANTS:-"--sort-role 0" "--sort-role 1 --sort-role-at 0" "--sort-role 1 --sort-role-at 1"}; do
      if [ "$cfg" = b256 ]; then a="--batch 256"; else a="--config $cfg"; fi
      tag=$(echo "$v" | tr -d ' -')
      $B $a $v --steps 300 --warmup 30 > "$OUT/sort_${cfg}_$tag.json" \
        2> "$OUT/sort_${cfg}_$tag.err" || exit $?
      python -c "import json;d=json.load(open('$OUT/sort_${cfg}_$tag.json'));print('$cfg $v',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
    done
  done
  ;;
flag)  # FLAG=--xyz: bench lines with $FLAG 0 and $FLAG 1 (CFGS)
  for cfg in ${CFGS:-terabyte kaggle b256}; do
    for val in 0 1; do
      if [ "$cfg" = b256 ]; then a="--batch 256"; else a="--config $cfg"; fi
      tag="${FLAG#--}_$val"
      $B $a $FLAG $val --steps 300 --warmup 30 > "$OUT/${cfg}_$tag.json" 2> "$OUT/${cfg}_$tag.err" \
        || exit $?
      python -c "import json;d=json.load(open('$OUT/${cfg}_$tag.json'));print('$cfg $FLAG $val',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
    done
  done
  ;;
tune)  # TUNE=key=value: bench lines without and with --tune $TUNE (CFGS)
  for cfg in ${CFGS:-terabyte kaggle b256}; do
    for on in 0 1; do
      if [ "$cfg" = b256 ]; then a="--batch 256"; else a="--config $cfg"; fi
      if [ $on = 1 ]; then t="--tune $TUNE"; else t=""; fi
      $B $a $t --steps 300 --warmup 30 > "$OUT/tune_${cfg}_$on.json" 2> "$OUT/tune_${cfg}_$on.err" \
        || exit $?
      python -c "import json;d=json.load(open('$OUT/tune_${cfg}_$on.json'));print('$cfg tune=$on $TUNE',d['value'],d['ms_per_step'],d['ms_per_step_p10_p50_p90'])"
    done
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
