set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r05_v36; mkdir -p $OUT
A="--s2m-modes= --odo= --map-keyframes 0 --pc2 0 --mapping= --allreduce-scans 0 --no-cpu --steps 20"
for n in 3 4 6 2 3; do
  timeout -k 10 200 python bench.py $A --streams $n > $OUT/s$n.json 2> $OUT/s$n.err || exit $?
  grep -h '^{' $OUT/s$n.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['ms_per_step'])" >> $OUT/summary.txt
done
