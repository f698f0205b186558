#!/bin/bash
# Retry a gpurun call while the pool reports no free box / infrastructure back-off (nothing ran,
# nothing charged); any other outcome (ok, a failing command, refusal) ends the loop.
#   bash tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && ! grep -q "run [1-9][0-9.]*s of limit" $LOG; then
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
