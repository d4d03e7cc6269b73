# training-step kernel traces of the in-tree library and an experiment library (same box)
set -o pipefail
mkdir -p gpurun_out
for LIB in tree "$@"; do
  if [ $LIB = tree ]; then unset WDMPNN_LIB; else export WDMPNN_LIB=$PWD/exp/libwdmpnn_$LIB.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_train_$LIB -o run --output-format csv -- python tools/train_bench.py > gpurun_out/train_$LIB.log 2>&1 || exit $?
  python tools/train_trace.py gpurun_out/rocprof_train_$LIB/run_kernel_trace.csv > gpurun_out/train_trace_$LIB.txt
  echo "== $LIB"; tail -1 gpurun_out/train_$LIB.log | cut -c1-200; tail -1 gpurun_out/train_trace_$LIB.txt
done
