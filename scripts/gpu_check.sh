#!/bin/bash
# One GPU session: parity tests, a short bench, and a rocprofv3 kernel-trace summary.
# Stops at the first step that faults / aborts / times out (exit codes >= 124 or signals).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >> "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name rc=$rc" >> "$OUT/steps.log"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${PROF:-1}" = 1 ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu
  python3 scripts/trace_prof_pass.py "$OUT/prof/run_kernel_trace.csv" 1 5 3 > "$OUT/prof_pass.json" 2>&1
fi
echo done >> "$OUT/steps.log"
