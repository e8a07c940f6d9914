#!/bin/bash
# Re-submit a gpurun call only when NOTHING ran (status=transient, or exit 3 = no box free).
# usage: tools/gpurun_retry.sh <timeout-seconds> '<command>'
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" > /tmp/gpurun_last.log 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_last.log || [ $rc -eq 3 ]; then
    echo "[retry] attempt $attempt: nothing ran (rc=$rc), waiting"; sleep 60; continue
  fi
  cat /tmp/gpurun_last.log; exit $rc
done
cat /tmp/gpurun_last.log; exit 3
