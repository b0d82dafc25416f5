#!/bin/bash
# Run GPU steps in order; stop at the first fault/abort/segfault/timeout
# (exit 124/134/137/139 or >128), continue past ordinary test failures (1).
# usage: tools/gpu_step.sh "<timeout_s> <logname> <cmd...>" ...   (shell quoting inside a step is honoured)
mkdir -p gpurun_out
rc_all=0
for step in "$@"; do
  eval set -- "$step"
  t=$1; log=$2; shift 2
  echo "=== [$log] timeout $t: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "=== [$log] rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$log"
  if [ $rc -ne 0 ]; then rc_all=$rc; fi
  if [ $rc -ge 124 ]; then echo "fault/timeout: stopping"; exit $rc; fi
done
exit $rc_all
