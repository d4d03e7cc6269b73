set -e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "one_launch or direct_training or golden" > gpurun_out/pytest_r5_v4.log 2>&1
timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/train_bench_v4.log 2>&1
STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/rocprof_train4 -o run -- python3 tools/train_bench.py > gpurun_out/train_prof_v4.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --stream-graphs 0 --stream-train-graphs 0 > gpurun_out/bench_sec_v6.log 2>&1
