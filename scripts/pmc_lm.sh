#!/bin/bash
# HBM traffic and SQ stall split of the two LM kernels (k_s2m_iter: configs[2] lm_applied leg;
# k_s2s_lm: the VLP-16 odometry leg), one counter group per rocprofv3 pass, kernel-trace only.
# The main leg runs at a small batch so the passes stay short.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc_lm}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu --streams 1 --batch 64 --prof-batches 1 --s2m-modes lm_applied --s2m-steps 2 --odo vlp16:1024 --allreduce-scans 0 --map-keyframes 0 --pc2 0 --mapping="
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || exit $?
python3 scripts/pmc_parse.py "$OUT" 1 > "$OUT/traffic.json"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS --kernel-trace --output-format csv -d "$PWD/$OUT/sq" -o run -- python3 bench.py $ARGS > "$OUT/sq.log" 2>&1 || exit $?
python3 scripts/pmc_sq.py "$OUT/sq" > "$OUT/sq.json"
