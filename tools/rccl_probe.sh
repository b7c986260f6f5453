#!/bin/bash
# One gpurun call: every rccl_capture_probe variant in its own process, each under its own
# time limit; stops at the first abort / fault / limit kill.  Logs: gpurun_out/r06/probe_*.log
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
for v in ${VARIANTS:-a2a_async a2a_splits g2_warm two_groups trainer g2_cold a2a_cold}; do
  for m in global thread_local; do
    timeout -k 10 90 python -u tools/rccl_capture_probe.py $v $m > gpurun_out/r06/probe_${v}_${m}.log 2>&1
    rc=$?
    echo "$v $m rc=$rc: $(grep RESULT gpurun_out/r06/probe_${v}_${m}.log | tail -1)"
    case $rc in 0|1) ;; 139) [ -n "$KEEP_GOING_ON_SEGV" ] || exit $rc;; *) echo "stopping after rc=$rc"; exit $rc;; esac
  done
done
