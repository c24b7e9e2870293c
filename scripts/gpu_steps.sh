#!/bin/bash
# Run GPU steps in order; each under its own time limit.  A step that ends in a fault, abort,
# segfault or timeout (rc not 0/1) stops the script; test failures (rc 1) do not.
# usage: scripts/gpu_steps.sh "name:seconds:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
