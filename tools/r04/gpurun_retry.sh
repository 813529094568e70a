#!/bin/bash
# gpurun with waits while no box is free (exit 3: nothing ran, nothing charged); any other exit is final
# usage: tools/r04/gpurun_retry.sh <log> <timeout> '<command>'
LOG=$1; TO=$2; shift 2
for i in $(seq 1 80); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && { echo "EXIT $rc" >> $LOG; exit $rc; }
  sleep 90
done
echo "EXIT 3 (gave up)" >> $LOG
