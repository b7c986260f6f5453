set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "tbe" > $O/pytest_tbe.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest_tbe.log
timeout -k 10 120 python tools/blas_ref.py > $O/blas_ref.txt 2>&1 || exit 1
cat $O/blas_ref.txt
timeout -k 10 120 python tools/ramp_probe.py --steps 1500 > $O/ramp0.txt 2>&1 || exit 1
timeout -k 10 120 python tools/ramp_probe.py --steps 1500 --preheat-ms 300 > $O/ramp300.txt 2>&1 || exit 1
cat $O/ramp0.txt $O/ramp300.txt
timeout -k 10 600 python tools/gemm_x6_ab.py --skip-acc --cfgs 128x128x2x4,128x128x4x2,64x64 --maths f32,x6 > $O/gemm_ab.txt 2>&1 || { tail $O/gemm_ab.txt; exit 1; }
cat $O/gemm_ab.txt
echo all-done
