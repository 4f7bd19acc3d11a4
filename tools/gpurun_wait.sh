#!/bin/bash
# usage: tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'  -- retries ONLY while gpurun reports no free box (transient)
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  rc=$?
  if grep -q "status=transient" $OUT; then sleep 90; continue; fi
  exit $rc
done
