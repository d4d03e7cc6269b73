set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "one_launch or direct_training or fp64 or random_graphs or training_step or golden" > gpurun_out/pytest_r5_v3.log 2>&1
WDMPNN_LIB=$PWD/exp/libwdmpnn_stamps.so timeout -k 10 120 python -u tools/stamps_small.py > gpurun_out/stamps_small_v2.log 2>&1
timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/train_bench_v3.log 2>&1
STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/rocprof_train -o run -- python3 tools/train_bench.py > gpurun_out/train_prof_v3.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --stream-graphs 0 --stream-train-graphs 0 > gpurun_out/bench_sec_v5.log 2>&1
