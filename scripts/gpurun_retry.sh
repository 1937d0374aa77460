#!/bin/bash
# Run one gpurun call; re-submit only when gpurun itself reports an infrastructure-side
# transient (box lost while being prepared / backing off / no box free), never after the
# command ran. Usage: scripts/gpurun_retry.sh <timeout> '<command>'
to=$1; shift
for attempt in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$to" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -qE "status=transient|backing off|no box|slot free|busy"; then
    sleep 60; continue
  fi
  exit $rc
done
exit 3
