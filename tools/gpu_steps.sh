#!/bin/bash
# Run GPU steps in order, each under its own time limit, output to gpurun_out/<name>.log.
#   tools/gpu_steps.sh "name|seconds|command" ...
# A step that fails with a test-failure status (1) does not stop the list; a fault, abort, segfault
# or time limit (any other non-zero status) ends the list: nothing more runs on the GPU after it.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "[steps] $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[steps] $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[steps] stopping after $name (rc $rc)"; exit $rc; fi
done
