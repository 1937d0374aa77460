#!/bin/bash
# HBM traffic per kernel from PMC counters, one counter group per rocprofv3 pass (FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass), kernel-trace only (no sys/runtime trace with --pmc). The
# bench runs 1 stream and no side legs so every dispatch is one whole batch of B scans.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}
B=${B:-1024}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu --streams 1 --batch $B --s2m-modes= --allreduce-scans 0 --odo= --map-keyframes 0 --pc2 0 --mapping="
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || exit $?
python3 scripts/pmc_parse.py "$OUT" "$B" > "$OUT/traffic.json"
# optional stall breakdown (8 SQ counters, one pass): where the wave cycles go per kernel
if [ "${SQ:-0}" = 1 ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --kernel-trace --output-format csv -d "$PWD/$OUT/sq" -o run -- python3 bench.py $ARGS > "$OUT/sq.log" 2>&1 || exit $?
  python3 scripts/pmc_sq.py "$OUT/sq" > "$OUT/sq.json"
fi
