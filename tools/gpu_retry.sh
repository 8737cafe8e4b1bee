#!/bin/bash
# Runs one gpurun call, again only while the pool has no box or slot for it
# (gpurun exit code 3: nothing ran, nothing charged). Any other result ends
# the loop. $1 = log file, $2 = gpurun --timeout, $3 = command, $4 = attempts.
log=$1; to=$2; cmd=$3; n=${4:-40}
for i in $(seq 1 "$n"); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
