#!/bin/bash
# Headline + HDL-64E odometry benches of the tree's library and of alternative builds
# (lego-loam-sr_amd/libllsr_<name>.so, names in LIBS), interleaved. Output under gpurun_out/$TAG.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab3}; mkdir -p "$OUT"
A="--odo ${ODO_LEGS:-hdl64e:512} --s2m-modes= --map-keyframes 0 --pc2 0 --mapping= --allreduce-scans 0 --no-cpu --steps 10"
for round in 1 2; do
  timeout -k 10 300 python bench.py $A > "$OUT/tree_$round.json" 2>/dev/null || exit $?
  for n in ${LIBS:?}; do
    LLSR_LIB=$PWD/lego-loam-sr_amd/libllsr_$n.so timeout -k 10 300 python bench.py $A > "$OUT/${n}_$round.json" 2>/dev/null || exit $?
  done
done
