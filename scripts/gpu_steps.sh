#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that faults,
# aborts or times out (exit >= 124), so nothing else touches the GPU after trouble.
# usage: scripts/gpu_steps.sh "<seconds>:<logname>:<command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  secs="${step%%:*}"; rest="${step#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc elapsed=$(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "stopping: $name exited with $rc"; exit $rc; fi
done
exit 0
