set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_stream.py tests/test_train_cli.py > gpurun_out/pytest_tnh2.log 2>&1
LIBS="tnx6 base" bash tools/r5_tn.sh > gpurun_out/tnh2_ab.txt 2>&1
LIBS="tnx6 base" bash tools/r5_tn.sh >> gpurun_out/tnh2_ab.txt 2>&1
