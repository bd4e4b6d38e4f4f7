#!/bin/bash
# usage: run.sh <logfile> <timeout> <command>; retries ONLY while gpurun reports no free slot (rc 3)
# (host-side helper: waits for a free GPU slot; never re-runs a command that ran)
log=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$cmd" > $log 2>&1
  rc=$?
  echo "rc=$rc try=$i" >> $log
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
