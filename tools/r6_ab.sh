# round 6: kernel stats (one batch in flight) of experiment libraries, stamps of the stamped one, and the
# driver's bench command per library (no CPU leg, no streamed training)
#   bash tools/r6_ab.sh "pairs5 ..." pstamps5
set -e
export TMPDIR=/tmp
D=gpurun_out/r6ab
mkdir -p $D
for v in $1; do
  export WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$v -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 ${AB_ARGS:-} > $D/prof_$v.log 2>&1
  python3 tools/kstats.py $D/prof_$v/run_kernel_stats.csv 5 > $D/kstats_$v.txt
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --stream-train-graphs 0 ${AB_ARGS:-} > $D/bench_$v.log 2>&1
done
if [ -n "$2" ]; then
  WDMPNN_LIB=$PWD/exp/libwdmpnn_$2.so timeout -k 10 300 python3 -u tools/stamps_layer.py > $D/stamps_$2.log 2>&1
fi
