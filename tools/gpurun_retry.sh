#!/bin/bash
# Retry a gpurun call only while the pool reports no free box / an
# infrastructure-side transient (gpurun exit code 3: nothing ran, nothing
# charged); any other outcome, including a failing command, ends it.
#   tools/gpurun_retry.sh <log> --timeout S -- '<command>'
log=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1; rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 100
done
exit 3
