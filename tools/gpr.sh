#!/bin/bash
# gpurun with retries while the pool has no free box / slot (exit 3 or a transient status);
# a refused, failed or finished call is returned as is.  Honours "retry in Ns" hints.
# usage: tools/gpr.sh <logfile> <timeout> <command>
LOG=$1; TO=$2; shift 2
rc=0
for i in $(seq 1 ${GPR_TRIES:-20}); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" "$LOG" && ! grep -q "status=ok" "$LOG"; }; then
    w=$(grep -o "retry in [0-9]*s" "$LOG" | tail -1 | grep -o "[0-9]*")
    sleep $(( ${w:-60} > 60 ? ${w:-60} + 5 : 75 ))
    continue
  fi
  exit $rc
done
exit $rc
