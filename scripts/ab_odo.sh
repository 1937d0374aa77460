#!/bin/bash
# A/B of the odometry legs: the tree's libllsr.so against lego-loam-sr_amd/libllsr_base.so (LLSR_LIB),
# after the LM parity tests on the tree's library. Output under gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
ODO="--odo ${ODO_LEGS:-hdl64e:512,vlp16:1024} --s2m-modes=${S2M_MODES:-} --map-keyframes 0 --pc2 0 --mapping=${MAPPING:-} --allreduce-scans 0 --no-cpu --steps ${STEPS:-5}"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_fa_lm.py tests/test_gpu_odometry.py} -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py $ODO > "$OUT/new.json" 2> "$OUT/new.err" || exit $?
LLSR_LIB=$PWD/lego-loam-sr_amd/libllsr_base.so timeout -k 10 300 python bench.py $ODO > "$OUT/base.json" 2> "$OUT/base.err" || exit $?
timeout -k 10 300 python bench.py $ODO > "$OUT/new2.json" 2> "$OUT/new2.err" || exit $?
