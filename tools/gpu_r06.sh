#!/bin/bash
# Round-6 GPU sessions (one stage per gpurun call):
#   bash tools/gpu_r06.sh tests   - pytest -m gpu (per-test timeout) + smoke()
#   bash tools/gpu_r06.sh bench   - default bench line + rocprofv3 kernel trace + PMC
#   bash tools/gpu_r06.sh configs - bench lines of C1 (small), C2 (kaggle), C4
set -o pipefail
STAGE=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${OUTNAME:-r06}
mkdir -p "$OUT"
cd "$ROOT" || exit 1
case $STAGE in
tests)
  # optional: K="expr" selects a subset (pytest -k)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider ${K:+-k "$K"} > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { tail -5 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  ;;
bench)
  timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
  tail -c 600 "$OUT/bench.json"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o kt \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 200 --warmup 20 \
    > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || exit $?
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-timing --no-graph --preheat-ms 0 --steps 10 \
      --warmup 2 > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err" || exit $?
  done
  echo "bench stage done"
  ;;
configs)
  for cfg in small kaggle terabyte_qr_rwsadagrad; do
    timeout -k 10 400 python bench.py --config $cfg > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" \
      || exit $?
    echo "$cfg: $(head -c 200 "$OUT/bench_$cfg.json")"
  done
  # the C3 widths at the W = 8 per-rank batch
  timeout -k 10 400 python bench.py --batch 256 > "$OUT/bench_b256.json" 2> "$OUT/bench_b256.err" \
    || exit $?
  echo "b256: $(head -c 200 "$OUT/bench_b256.json")"
  ;;
esac
# (pmc only: bash tools/gpu_r06.sh pmc)
if [ "$STAGE" = pmc ]; then
  cd /tmp && export TMPDIR=/tmp
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc \
      -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-kernel-timing --no-graph --preheat-ms 0 \
      --steps 10 --warmup 2 > "$OUT/pmc_$C.json" 2> "$OUT/pmc_$C.err" || exit $?
  done
  echo "pmc stage done"
fi
# emulated W = 8 ranks (one GPU): bash tools/gpu_r06.sh emulate
if [ "$STAGE" = emulate ]; then
  for R in ${RANKS:-2 0}; do
    timeout -k 10 400 python bench.py ${ECFG:+--config $ECFG} --emulate-world 8 --emulate-rank $R \
      --emulate-capture ${ECAP:-segments} --steps 300 --no-cpu-baseline \
      > "$OUT/bench_emul8${ECFG:+_$ECFG}_${ECAP:-segments}_r$R.json" \
      2> "$OUT/bench_emul8_r$R.err" || exit $?
    echo "rank $R: $(head -c 300 "$OUT/bench_emul8${ECFG:+_$ECFG}_${ECAP:-segments}_r$R.json")"
  done
  timeout -k 10 400 python bench.py --batch 256 --no-cpu-baseline --steps 300 \
    > "$OUT/bench_b256.json" 2> "$OUT/bench_b256.err" || exit $?
  echo "b256: $(head -c 200 "$OUT/bench_b256.json")"
fi
# per-shape GEMM table vs hipBLASLt: bash tools/gpu_r06.sh blas
if [ "$STAGE" = blas ]; then
  GEMM_VS_BLAS_OUT="$OUT/gemm_vs_blas.json" timeout -k 10 300 python -u tools/gemm_vs_blas.py ${BATCHES:-2048 256} \
    > "$OUT/gemm_vs_blas.txt" 2>&1 || { tail -5 "$OUT/gemm_vs_blas.txt"; exit 1; }
  tail -3 "$OUT/gemm_vs_blas.txt"
fi
# GEMM investigation: per-shape table vs hipBLASLt, hipBLASLt's kernel names (tile config), and
# SQ counters of one C3 shape (library launch, lab cfgs, torch.mm): bash tools/gpu_r06.sh gemmprobe
if [ "$STAGE" = gemmprobe ]; then
  GEMM_VS_BLAS_OUT="$OUT/gemm_vs_blas.json" timeout -k 10 300 python -u tools/gemm_vs_blas.py 2048 256 \
    > "$OUT/gemm_vs_blas.txt" 2>&1 || { tail -5 "$OUT/gemm_vs_blas.txt"; exit 1; }
  tail -3 "$OUT/gemm_vs_blas.txt"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/blas_kt" -o kt \
    -- python3 "$ROOT/tools/gemm_vs_blas.py" 2048 --blas-only > "$OUT/blas_kt.txt" 2>&1 || exit $?
  for SH in fwd1 wgrad1; do
    P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
    timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/pmc_$SH" -o p1 \
      -- python3 "$ROOT/tools/gemm_pmc_probe.py" $SH 101,105 > "$OUT/pmc_$SH.txt" 2>&1 || exit $?
    P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE"
    timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/pmc2_$SH" -o p2 \
      -- python3 "$ROOT/tools/gemm_pmc_probe.py" $SH 101,105 > "$OUT/pmc2_$SH.txt" 2>&1 || exit $?
  done
  echo "gemmprobe done"
fi
# W > 1 tail A/B (emulated W = 8, segment capture): bash tools/gpu_r06.sh emulab
if [ "$STAGE" = emulab ]; then
  for R in ${RANKS:-2}; do
    for TR in 0 1 0 1; do
      timeout -k 10 300 python bench.py ${ECFG:+--config $ECFG} --emulate-world 8 --emulate-rank $R \
        --tbe-role $TR --steps 300 --no-cpu-baseline --no-kernel-timing \
        > "$OUT/emulab${ECFG:+_$ECFG}_r${R}_tr$TR.json" 2> "$OUT/emulab_r$R.err" || exit $?
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1].split('/')[-1], d['emulated'].get('ms_per_step', d.get('ms_per_step')), d['ms_per_step_p10_p50_p90'])" \
        "$OUT/emulab${ECFG:+_$ECFG}_r${R}_tr$TR.json"
    done
  done
fi
# bottom-MLP parts A/B at C3: bash tools/gpu_r06.sh partsab
if [ "$STAGE" = partsab ]; then
  for i in 1 2; do
    for P in 0 2; do
      timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --steps 300 --bottom-parts $P \
        > "$OUT/parts$P_$i.json" 2> "$OUT/parts.err" || exit $?
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('parts $P', d['value'], d['ms_per_step'], d['ms_per_step_p10_p50_p90'])" "$OUT/parts$P_$i.json" | tee -a "$OUT/partsab.txt"
    done
  done
fi
# one-step kernel timelines: bash tools/gpu_r06.sh trace
if [ "$STAGE" = trace ]; then
  bash tools/step_trace.sh gpurun_out/${OUTNAME:-r06}/trace_c3 || exit $?
  bash tools/step_trace.sh gpurun_out/${OUTNAME:-r06}/trace_b256 --batch 256 || exit $?
  bash tools/step_trace.sh gpurun_out/${OUTNAME:-r06}/trace_kaggle --config kaggle || exit $?
fi
