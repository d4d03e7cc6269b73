# parity tests + short streamed bench on an experiment library (LIB)
set -o pipefail
mkdir -p gpurun_out
export WDMPNN_LIB=$PWD/exp/libwdmpnn_${LIB:-np}.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread --deselect tests/test_gpu_parity.py::test_native_library_is_the_code_that_runs > gpurun_out/pytest_$LIB.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_$LIB.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-secondary --stream-graphs 200000 --stream-train-graphs 65536 > gpurun_out/bench_$LIB.log 2>&1 || exit $?
python -c "
import json,sys; l=[x for x in open('gpurun_out/bench_$LIB.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$LIB', 'streamed', round(d['streamed']['value']/1e6,1), 'stream-train ms', round(d['streamed_training']['ms_per_step'],3))"
done
