#!/bin/bash
# HBM traffic per kernel from PMC counters, one counter group per rocprofv3 pass (FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass), kernel-trace only (no sys/runtime trace with --pmc).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 4 --warmup 1 --no-cpu --streams 1"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || exit $?
python3 scripts/pmc_parse.py "$OUT" > "$OUT/traffic.json"
