#!/usr/bin/env bash
# Run GPU steps under per-step time limits. A plain failure (exit 1-123) is recorded and
# the next step runs; a timeout, abort or crash (exit >= 124) ends the script at once so
# nothing else touches a possibly-faulted GPU.
# usage: tools/gpu_steps.sh "SECONDS|LOGNAME|command" ...
set -u
mkdir -p gpurun_out
status=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ "$rc" -ge 124 ]; then
    echo "FATAL: step $name ended with rc=$rc; stopping"
    exit "$rc"
  fi
  [ "$rc" -ne 0 ] && status=1
done
exit $status
