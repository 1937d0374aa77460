#!/bin/bash
# Run one gpurun call; re-submit only when gpurun itself reports an infrastructure-side
# transient (box lost while being prepared / backing off / no box free), never after the
# command ran. Usage: LOG=/tmp/x.log scripts/gpurun_retry.sh <timeout> '<command>'
to=$1; shift
log=${LOG:-/tmp/gpurun_retry.log}
for attempt in $(seq 1 ${ATTEMPTS:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1; rc=$?
  if grep -qE "status=transient|backing off|no box|slot free|busy" "$log" && ! grep -q "status=ok\|status=fail" "$log"; then
    sleep ${WAIT:-90}; continue
  fi
  tail -30 "$log"
  exit $rc
done
exit 3
