#!/bin/bash
# Headline-only bench over batch sizes x stream counts (BATCHES, STREAMS), one line per run in
# gpurun_out/$TAG/summary.txt: batch streams value ms_per_step k_vox_pcl_ms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bsweep}; mkdir -p "$OUT"
A="--s2m-modes= --odo= --map-keyframes 0 --pc2 0 --mapping= --allreduce-scans 0 --no-cpu --steps 20"
for b in ${BATCHES:-1024 2048 4096}; do
  for n in ${STREAMS:-3}; do
    timeout -k 10 200 python bench.py $A --batch $b --streams $n > "$OUT/b${b}_s$n.json" 2> "$OUT/b${b}_s$n.err" || exit $?
    grep -h '^{' "$OUT/b${b}_s$n.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, $n, d['value'], d['ms_per_step'], d['kernels_ms_per_step']['k_vox_pcl'])" >> "$OUT/summary.txt"
  done
done
cat "$OUT/summary.txt"
