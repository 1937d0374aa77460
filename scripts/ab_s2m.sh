#!/bin/bash
# Scan-to-map legs (lm_applied, faithful) of the tree's library and of variants
# lego-loam-sr_amd/libllsr_<name>.so (LIBS), interleaved twice. Output under gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abs2m}; mkdir -p "$OUT"
A="--no-cpu --odo= --map-keyframes 0 --pc2 0 --mapping= --allreduce-scans 0 --steps 3 --warmup 1 --batch 512"
for round in 1 2; do
  timeout -k 10 300 python bench.py $A > "$OUT/tree_$round.json" 2>"$OUT/tree_$round.err" || exit $?
  for n in ${LIBS:?}; do
    LLSR_LIB=$PWD/lego-loam-sr_amd/libllsr_$n.so timeout -k 10 300 python bench.py $A > "$OUT/${n}_$round.json" 2>"$OUT/${n}_$round.err" || exit $?
  done
done
