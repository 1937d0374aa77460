#!/bin/bash
# configs[1] leg only (other legs skipped): scans/s for a few (batch, streams) pairs.
set -u
mkdir -p gpurun_out/sweep
A="--no-cpu --s2m-modes= --allreduce-scans 0 --odo= --map-keyframes 0 --pc2 0 --steps 20"
for cfg in ${SWEEP:-"1024:3" "1024:4" "1024:2" "2048:3" "2048:4" "1536:3"}; do
  b=${cfg%%:*}; st=${cfg##*:}
  timeout -k 10 200 python bench.py $A --batch $b --streams $st > gpurun_out/sweep/b${b}_s${st}.log 2>&1 || exit $?
done
