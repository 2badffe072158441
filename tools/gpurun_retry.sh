#!/bin/bash
# gpurun with retries ONLY for infrastructure transients (no box / box taken
# away before the command ran: gpurun status "transient" or exit code 3; nothing
# ran, nothing charged).  A command that ran and failed is never retried.
#   tools/gpurun_retry.sh <logfile> <timeout> '<command>'
log=$1; to=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "transient (attempt $i), retrying" >> "$log.retries"; sleep 200; continue
  fi
  exit $rc
done
exit 3
