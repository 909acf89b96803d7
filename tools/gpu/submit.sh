#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool reports no free
# slot / box (exit 3 or a "transient" status: nothing ran, nothing charged).
#   tools/gpu/submit.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then sleep 90; continue; fi
  exit $rc
done
exit 3
