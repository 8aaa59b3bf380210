#!/bin/bash
# retry gpurun while it reports exit 3 (no box / slot free; nothing ran, nothing charged)
LOG=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  echo "exit $rc (attempt $i)" >> $LOG
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
