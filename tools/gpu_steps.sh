#!/bin/bash
# Run GPU steps in order; each under its own time limit. Stop at the first fault-like exit
# (abort/segfault/timeout/kill) — an ordinary test failure (exit 1) does not stop the chain.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)"; tail -n 15 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "=== stopping after $name (rc=$rc)"; exit $rc ;;
  esac
done
