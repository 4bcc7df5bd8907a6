#!/bin/bash
# Runs GPU steps in order, each under its own time limit.  A step that ends in
# a crash (signal / abort / timeout: rc >= 2 for pytest, or >= 124) stops the
# sequence so nothing else touches a possibly faulted GPU.  Plain test
# failures (pytest rc 1) do not stop later steps.
#   tools/gpu_run.sh "name:timeout:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "== $name (limit ${to}s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping after $name (rc=$rc)"
    exit $rc
  fi
done
exit 0
