#!/bin/bash
# gpurun_bg.sh LOG TIMEOUT CMD... : one gpurun call; only when NO box/slot was available
# (exit 3: nothing ran, nothing charged) it is made again after 3 minutes, up to 8 times.
LOG=$1; TO=$2; shift 2
for i in $(seq 1 ${ATTEMPTS:-8}); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  echo "EXIT $rc" >> $LOG
  [ $rc -ne 3 ] && exit $rc
  sleep 180
done
