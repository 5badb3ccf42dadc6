#!/bin/bash
# Helpers for GPU-box scripts: run one GPU step under its own time limit; stop the script on a
# timeout, crash or abort (exit >= 124, or a signal), go on after ordinary failures (1, 2).
#   source tools/gpu_step.sh; step NAME SECONDS cmd...
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -4 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
  return 0
}
