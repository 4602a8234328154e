#!/bin/bash
# Submit one gpurun call; resubmit only when the box could not be prepared ("status=transient")
# or no slot was free (exit 3).  A command that ran and failed is never resubmitted.
# usage: tools/gpu.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 ${GPU_TRIES:-30}); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1); rc=$?
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then
    echo "[gpu.sh] attempt $i: box not ready, waiting" >&2; sleep 90; continue
  fi
  echo "$out"; exit $rc
done
echo "$out"; exit 1
