set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "full_schedule" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
bash tools/ab_env.sh $O "DLRM_BOT_SCHED=partial" "DLRM_BOT_SCHED=full" "DLRM_BOT_SCHED=partial DLRM_FULL_LAST_WGRAD=1"
