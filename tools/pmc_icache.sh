#!/bin/bash
# Instruction-fetch cost of one GEMM shape (tools/gemm_one.py): wave-cycle breakdown, VALU /
# MFMA instruction counts and SQC instruction-cache hits / misses, each in its own
# rocprofv3 --pmc pass.  Usage: bash tools/pmc_icache.sh <tag> <gemm_one.py args...>
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES"
timeout -s KILL 60 rocprofv3 --pmc $P1 --output-format csv -d "$OUT/i1" -o i1 \
  -- python3 "$ROOT/tools/gemm_one.py" "$@" > "$OUT/i1.txt" 2>&1 || exit $?
P2="SQC_ICACHE_MISSES SQC_ICACHE_HITS"
timeout -s KILL 60 rocprofv3 --pmc $P2 --output-format csv -d "$OUT/i2" -o i2 \
  -- python3 "$ROOT/tools/gemm_one.py" "$@" > "$OUT/i2.txt" 2>&1 || exit $?
grep TF "$OUT/i2.txt"
