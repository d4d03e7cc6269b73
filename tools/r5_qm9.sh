set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "one_launch or blocked_fused or golden" > gpurun_out/pytest_qm9.log 2>&1
WDMPNN_LIB=$PWD/exp/libwdmpnn_stamps.so timeout -k 10 120 python -u tools/stamps_small.py > gpurun_out/stamps_small_v3.log 2>&1
timeout -k 10 200 python -u tools/qm9_streams.py > gpurun_out/qm9_streams_v2.log 2>&1
