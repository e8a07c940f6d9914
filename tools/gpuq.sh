#!/bin/bash
# queue a gpurun call: retry ONLY while no box/slot was available (nothing ran, nothing charged)
out=$1; shift
for i in $(seq 1 40); do
  timeout 2700 /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  if grep -q 'status=transient' "$out" && ! grep -q 'status=ok\|status=fail\|status=error' "$out"; then
    sleep 90; continue
  fi
  echo "rc=$rc tries=$i" >> "$out"; exit $rc
done
echo "gave up" >> "$out"
