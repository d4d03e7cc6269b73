# ad-hoc GPU session: parity tests on an experiment library, kernel stats, same-box A/B against others
set -o pipefail
mkdir -p gpurun_out
LIB=${LIB:-ws}
WDMPNN_LIB=$PWD/exp/libwdmpnn_$LIB.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread --deselect tests/test_gpu_parity.py::test_native_library_is_the_code_that_runs > gpurun_out/pytest_$LIB.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_$LIB.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh $LIB || exit $?
timeout -k 10 600 bash tools/ab3.sh $LIB ${AB:-cur} || exit $?
