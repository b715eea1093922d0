#!/bin/bash
# Run GPU steps in order, each under its own time limit. A step that ends with
# a plain failure (exit 1: assertion / test failure / Python exception) does not
# stop the sequence; anything else (timeout 124/137, abort 134, segfault 139,
# GPU fault) stops it so nothing more touches the GPU in this call.
# usage: tools/gpu_steps.sh "<secs>|<logname>|<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; log="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$log] $cmd (limit ${secs}s)"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "=== [$log] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 5 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping: rc=$rc"; exit $rc; fi
done
exit 0
