#!/bin/bash
# gpurun with retries while no box / slot is free (exit code 3 only); $1 = log, rest = gpurun args
LOG=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 60
done
echo "rc=$rc tries=$i" >> $LOG
