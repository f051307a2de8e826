#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# crash-like exit (fault/abort/segfault/timeout), continue past ordinary test
# failures (exit 1) so later measurements still run.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0|1|5) ;;
    *) echo "=== stopping: step $name exited $rc"; exit $rc ;;
  esac
done
