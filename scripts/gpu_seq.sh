#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first failure, and treat a
# runtime fault message in a step's log as a failure even when the step exited 0.
#   TAG=r06_vN bash scripts/gpu_seq.sh "name|timeout|cmd" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-seq}
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "== $name" >> "$OUT/steps.log"
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  if grep -q "HSA_STATUS_ERROR\|illegal memory access" "$OUT/$name.log"; then rc=99; fi
  echo "rc=$rc" >> "$OUT/steps.log"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name rc=$rc"; exit $rc; fi
done
echo done >> "$OUT/steps.log"
