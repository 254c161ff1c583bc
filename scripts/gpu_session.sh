#!/bin/bash
# Run a sequence of GPU steps on the gpurun box, each under its own time limit. A step that ends
# in a crash/abort/timeout (exit >= 124, or a signal) stops the script: nothing else touches the
# GPU after a fault. Ordinary failures (exit 1/2, e.g. failing tests) do not stop later steps.
#   usage: scripts/gpu_session.sh "<name>|<seconds>|<command>" ...
set -u
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping: step $name ended with $rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
  [ $rc -ne 0 ] && status=$rc
done
exit $status
