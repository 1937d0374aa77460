#!/bin/bash
# A/B of the headline (configs[1] IP + features): the tree's libllsr.so against
# lego-loam-sr_amd/libllsr_base.so (LLSR_LIB), after parity tests (TESTS) on the tree's library.
# Output under gpurun_out/$TAG. Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abh}
mkdir -p "$OUT"
H="--no-cpu --s2m-modes= --odo= --map-keyframes 0 --pc2 0 --mapping= --allreduce-scans 0 ${BENCH_ARGS:-}"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v -m gpu -x --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit $?
fi
timeout -k 10 200 python bench.py $H > "$OUT/new.json" 2> "$OUT/new.err" || exit $?
LLSR_LIB=$PWD/lego-loam-sr_amd/libllsr_base.so timeout -k 10 200 python bench.py $H > "$OUT/base.json" 2> "$OUT/base.err" || exit $?
timeout -k 10 200 python bench.py $H > "$OUT/new2.json" 2> "$OUT/new2.err" || exit $?
