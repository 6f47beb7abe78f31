#!/bin/bash
# Run GPU steps in sequence; stop at the first crash/timeout (exit >= 124 or
# signal), continue past ordinary test failures (exit 1).  Logs in gpurun_out/.
mkdir -p gpurun_out
step() {   # step <name> <timeout-seconds> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
