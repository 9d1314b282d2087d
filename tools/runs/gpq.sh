#!/bin/bash
# Queue one gpurun call: retry while the pool has no free box (status=transient,
# nothing charged); any other outcome ends the loop.  Usage:
#   tools/runs/gpq.sh LOGFILE TIMEOUT 'command'
log=$1; to=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log"; then sleep 45; continue; fi
  echo "rc=$rc" >> "$log"
  exit $rc
done
echo "gave up: no box" >> "$log"
