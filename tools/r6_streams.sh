# round 6: batches in flight for the polymer headline, same box (--streams 2 / 3 / 4 / 5, driver command without the CPU leg and secondaries)
set -e
export TMPDIR=/tmp
D=gpurun_out/r6st
mkdir -p $D
for n in 3 4 2 5 3 4; do
  echo "== streams $n" >> $D/streams.log
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu --no-secondary --many 0 --stream-graphs 0 --stream-train-graphs 0 --streams $n >> $D/streams.log 2>&1
done
