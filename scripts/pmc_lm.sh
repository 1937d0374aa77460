#!/bin/bash
# HBM traffic and SQ stall split of the LM kernels, one counter group per rocprofv3 pass,
# kernel-trace only: leg A = the configs[2] scan-to-map lm_applied leg (k_s2m_iter / k_s2m_solve,
# P = 256) + the VLP-16 odometry leg (k_s2s_lm, 1024 scans); leg B = the HDL-64E odometry leg
# (k_s2s_lm, 512 scans). The IP leg runs at a small batch so the passes stay short.
# Output: $OUT/traffic_lm.json (scripts/pmc_lm_merge.py), the format of profiles/traffic_lm_latest.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc_lm}
mkdir -p "$OUT"
export TMPDIR=/tmp
COMMON="--steps 1 --warmup 1 --no-cpu --streams 1 --batch 64 --prof-batches 1 --s2m-steps 2 --allreduce-scans 0 --map-keyframes 0 --pc2 0 --mapping="
ARGS_A="$COMMON --s2m-modes lm_applied --odo vlp16:1024"
ARGS_B="$COMMON --s2m-modes= --odo hdl64e:512"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS"
for leg in A B; do
  if [ $leg = A ]; then ARGS=$ARGS_A; else ARGS=$ARGS_B; fi
  mkdir -p "$OUT/$leg"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/$leg/fetch" -o run -- python3 bench.py $ARGS > "$OUT/$leg/fetch.log" 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/$leg/write" -o run -- python3 bench.py $ARGS > "$OUT/$leg/write.log" 2>&1 || exit $?
  python3 scripts/pmc_parse.py "$OUT/$leg" 1 > "$OUT/$leg/traffic.json" || exit $?
  timeout -s KILL 300 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d "$PWD/$OUT/$leg/sq" -o run -- python3 bench.py $ARGS > "$OUT/$leg/sq.log" 2>&1 || exit $?
  python3 scripts/pmc_sq.py "$OUT/$leg/sq" > "$OUT/$leg/sq.json" || exit $?
done
python3 scripts/pmc_lm_merge.py "$OUT" "${SRC:-$OUT}" > "$OUT/traffic_lm.json"
