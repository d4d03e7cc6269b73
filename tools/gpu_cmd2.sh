set -o pipefail
mkdir -p gpurun_out
export WDMPNN_LIB=$PWD/exp/libwdmpnn_gb.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread --deselect tests/test_gpu_parity.py::test_native_library_is_the_code_that_runs > gpurun_out/pytest_gb.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-secondary --stream-graphs 200000 --stream-train-graphs 65536 > gpurun_out/bench_gb.log 2>&1 || exit $?
unset WDMPNN_LIB
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-secondary --stream-graphs 200000 --stream-train-graphs 65536 > gpurun_out/bench_tree.log 2>&1 || exit $?
for f in gb tree; do python -c "
import json,sys; l=[x for x in open('gpurun_out/bench_$f.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$f', 'streamed', round(d['streamed']['value']/1e6,1), 'stream-train ms', round(d['streamed_training']['ms_per_step'],3))"; done
export WDMPNN_LIB=$PWD/exp/libwdmpnn_gb.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_gb -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu --no-secondary --stream-graphs 0 --stream-train-graphs 0 > gpurun_out/rocprof_gb.log 2>&1 || exit $?
python tools/kstats.py gpurun_out/rocprof_gb/run_kernel_stats.csv 8 | grep graph_build
