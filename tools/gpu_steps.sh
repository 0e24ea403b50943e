#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit.  A step that fails
# normally (exit 1/2: test failure, python error) does not stop the chain;
# a fault, abort, segfault or timeout (124, 134, 137, 139, >128) ends the call.
#
# usage: tools/gpu_steps.sh "<secs>|<name>|<command>" ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"
  name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  end=$(date +%s)
  echo "=== [$name] rc=$rc in $((end-start))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] ; then
    echo "=== stopping: step $name ended with rc=$rc (fault/timeout)"
    exit $rc
  fi
done
exit 0
