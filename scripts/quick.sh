#!/bin/bash
# A short GPU iteration: selected parity tests, a phase profile, and a headline-only bench.
#   TAG=r03_vN TESTS="tests/test_gpu_parity.py ..." PHASES="8:-2:8" BENCH_ARGS="..." bash scripts/quick.sh
# Stops at the first step that faults / aborts / times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-quick}
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >> "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name rc=$rc" >> "$OUT/steps.log"; exit $rc; fi
}
if [ -n "${TESTS:-}" ]; then
  step pytest 600 python -u -m pytest $TESTS -v -m gpu -x --timeout 120 --timeout-method thread
fi
if [ -n "${PHASES:-}" ]; then
  PHASES=$PHASES step phase 300 python -u scripts/phase_profile.py ${PHASE_LIDAR:-vlp16} ${PHASE_B:-1024}
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench 600 python -u bench.py --no-cpu --s2m-modes "" --odo "" --map-keyframes 0 --pc2 0 --mapping "" \
    --allreduce-scans 0 ${BENCH_ARGS:-}
fi
if [ -n "${EXTRA:-}" ]; then
  step extra 600 bash -c "$EXTRA"
fi
echo done >> "$OUT/steps.log"
