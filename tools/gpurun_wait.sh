#!/bin/bash
# Run one gpurun call, re-submitting it only while the pool reports that no box was available
# (status=transient with nothing run or charged); any call whose command ran -- pass or fail --
# ends the loop.  usage: bash tools/gpurun_wait.sh TIMEOUT 'command'
T=$1; shift
for attempt in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  echo "$out" | grep -v amdgpu.ids | tail -${GW_TAIL:-25}
  if echo "$out" | grep -q "status=transient" && echo "$out" | grep -qE "run 0\.0s|run Nones"; then
    echo "[gpurun_wait] attempt $attempt: no box; waiting"
    sleep 150
    continue
  fi
  exit 0
done
echo "[gpurun_wait] gave up"
