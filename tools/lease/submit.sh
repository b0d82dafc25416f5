#!/bin/bash
# Submit one lease script through gpurun, re-submitting only when no box was
# obtained (exit 3: no box free; or a transient infrastructure event before the
# command ran).  A command that ran -- whatever its exit status -- is never re-run.
# usage: tools/lease/submit.sh <lease script> <out file> [timeout_s]
script=$1; out=$2; to=${3:-1200}
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "bash $script" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 200; continue; fi
  exit $rc
done
exit 3
