#!/bin/bash
# Run one gpurun call, retrying ONLY while the pool has no free slot or box
# (gpurun exit 3, or its "transient" status: nothing ran, nothing charged).
# Any other outcome -- success or a failure of the command itself -- ends it.
# Usage: tools/gpu_retry.sh <log> <timeout_s> <command>
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    sleep 90
    continue
  fi
  echo "gpurun rc=$rc after $i tries" >> "$log"
  exit $rc
done
echo "gave up: no slot" >> "$log"
exit 3
