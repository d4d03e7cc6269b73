set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_forward_many.py tests/test_atom_blocks.py > gpurun_out/pytest_host.log 2>&1
timeout -k 10 200 python -u tools/host_breakdown.py > gpurun_out/host_breakdown_v3.log 2>&1
timeout -k 10 200 python -u tools/short_run.py > gpurun_out/short_run_v5.log 2>&1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_host_20.log 2>&1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu > gpurun_out/bench_host_200.log 2>&1
