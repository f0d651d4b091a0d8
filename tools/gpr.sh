#!/bin/bash
# (dev helper) gpurun with retries while no slot is free (exit 3 / transient); never retries a command that ran.
out=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient\|rc=None" $out && ! grep -q "run [1-9][0-9.]*s of limit" $out; then sleep 120; continue; fi
  exit $rc
done
exit $rc
