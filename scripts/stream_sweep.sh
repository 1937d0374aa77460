set -u
mkdir -p gpurun_out/sweep
A="--no-cpu --s2m-modes= --allreduce-scans 0 --odo= --map-keyframes 0 --pc2 0 --steps 20"
for cfg in "1024 3" "1024 4" "1024 2" "2048 3" "2048 2" "512 4"; do
  set -- $cfg
  timeout -k 10 200 python bench.py $A --batch $1 --streams $2 > gpurun_out/sweep/b$1_s$2.log 2>&1 || exit $?
done
