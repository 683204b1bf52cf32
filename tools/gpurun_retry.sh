#!/bin/bash
# Development helper: run one gpurun call, retrying only while the pool has no free slot / box
# (exit 3 or a transient infrastructure status — nothing ran, nothing was charged).
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient\|no free box\|are busy\|backing off" "$log" && ! grep -q "status=ok" "$log"; then
    sleep 60; continue
  fi
  exit $rc
done
exit 3
