#!/bin/bash
# PMC passes on one GEMM (ours and hipBLASLt) -> gpurun_out/pmc_gemm/
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_gemm
SHAPE=${1:-2048,1024,1028,0,1}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
for who in ours blas; do
  for i in 1 2; do
    eval P=\$P$i
    if [ $who = blas ]; then export GEMM_ONE_BLAS=1; else unset GEMM_ONE_BLAS; fi
    timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/${who}_$i -o p -- python3 $ROOT/tools/gemm_one.py $SHAPE 10 > $OUT/${who}_$i.log 2>&1 || exit $?
  done
done
echo done
