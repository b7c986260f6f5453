#!/bin/bash
# gpurun with retries on "no box / slot free" (exit 3) or transient infra status only
# usage: tools/gpr.sh <logfile> <timeout> <command>
LOG=$1; TO=$2; shift 2
for i in $(seq 1 ${GPR_TRIES:-20}); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|slot(s) on this pod are busy\|backing off" "$LOG" && ! grep -q "status=ok" "$LOG"; then
    sleep 75; continue
  fi
  [ $rc -eq 3 ] && { sleep 75; continue; }
  exit $rc
done
exit $rc
