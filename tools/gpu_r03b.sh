set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "alloc or c3_table_list or index_error or c1_full or deferred" > $O/pytest_fix.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest_fix.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench rc=$?; tail -20 $O/bench_default.err; exit 1; }
tail -c 3000 $O/bench_default.json
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driverlike.json 2> $O/bench_driverlike.err || exit 1
for cfg in small kaggle; do
  timeout -k 10 400 python bench.py --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { echo $cfg rc=$?; tail -20 $O/bench_$cfg.err; exit 1; }
done
for lr in 0.1 0.01; do
  timeout -k 10 300 python bench.py --config terabyte_qr_rwsadagrad --lr $lr --no-cpu-baseline --no-kernel-timing --steps 300 > $O/bench_c4_lr$lr.json 2> $O/bench_c4_lr$lr.err || exit 1
done
echo all-done
