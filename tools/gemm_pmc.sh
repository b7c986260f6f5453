#!/bin/bash
# MFMA utilisation / stall breakdown of one GEMM shape (tools/gemm_one.py) from rocprofv3
# PMC passes.  Usage: bash tools/gemm_pmc.sh <tag> <gemm_one.py args...>
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt \
  -- python3 "$ROOT/tools/gemm_one.py" "$@" > "$OUT/kt.txt" 2>&1 || exit $?
grep TF "$OUT/kt.txt"
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/p1" -o p1 \
  -- python3 "$ROOT/tools/gemm_one.py" "$@" > "$OUT/p1.txt" 2>&1 || exit $?
echo done1
P2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_UNALIGNED_STALL"
timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/p2" -o p2 \
  -- python3 "$ROOT/tools/gemm_one.py" "$@" > "$OUT/p2.txt" 2>&1 || exit $?
echo done2
