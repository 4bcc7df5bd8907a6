#!/bin/bash
# retry a gpurun call only while the pool reports no box / transient (rc 3); logs to $1
log=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1; rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 100
done
exit 3
