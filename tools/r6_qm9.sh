# round 6: QM9-sized batches in flight (the one-launch small forward), same box: --streams 1 / 2 / 4 / 8, and the
# rocprofv3 kernel stats of the four-stream run (kernel time under concurrency)
set -e
export TMPDIR=/tmp
D=gpurun_out/r6q9
mkdir -p $D
for n in 1 2 4 8 4; do
  echo "== streams $n" >> $D/streams.log
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu --no-secondary --many 0 --stream-graphs 0 --stream-train-graphs 0 --kind qm9 --streams $n >> $D/streams.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof4 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --many 0 --stream-graphs 0 --stream-train-graphs 0 --kind qm9 --streams 4 > $D/prof4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof1 -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --many 0 --stream-graphs 0 --stream-train-graphs 0 --kind qm9 --streams 1 > $D/prof1.log 2>&1
python3 tools/kstats.py $D/prof4/run_kernel_stats.csv 3 > $D/kstats4.txt
python3 tools/kstats.py $D/prof1/run_kernel_stats.csv 3 > $D/kstats1.txt
