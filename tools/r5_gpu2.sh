set -e
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "direct or training or golden or random or grad" > gpurun_out/pytest_r5_v5.log 2>&1
timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/train_bench_v5.log 2>&1
STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/rocprof_train5 -o run -- python3 tools/train_bench.py > gpurun_out/train_prof_v5.log 2>&1
SAB_TAG=_p4 bash tools/stream_ab_libs.sh base nogroup > gpurun_out/sab_p4.txt 2>&1
SAB_TAG=_p2 SAB_ARGS="--producers 2" bash tools/stream_ab_libs.sh base nogroup > gpurun_out/sab_p2.txt 2>&1
