set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest.log; grep FAILED $O/pytest.log | head -20
bash tools/ab_env.sh $O "DLRM_GEMM_BODY=dma" "DLRM_GEMM_BODY=reg"
