# rocprof kernel stats of the single-stream bench for each experiment library named
set -o pipefail
mkdir -p gpurun_out
for LIB in "$@"; do
  WDMPNN_LIB=$PWD/exp/libwdmpnn_$LIB.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_$LIB -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 > gpurun_out/rocprof_$LIB.log 2>&1 || exit $?
  echo "== $LIB"; python tools/kstats.py gpurun_out/rocprof_$LIB/run_kernel_stats.csv 4
done
