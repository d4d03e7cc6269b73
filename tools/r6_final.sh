# round 6 final evidence on one box: the GPU suite, smoke, the driver's bench command next to a 200-step run,
# and the same command restricted to two CPUs
set -e
export TMPDIR=/tmp
D=gpurun_out/r6z
mkdir -p $D
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $D/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1
{ echo '$ python3 bench.py --gpus 1 --steps 20 --warmup 5'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5;
  echo '$ python3 bench.py --gpus 1 --steps 200 --warmup 20'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 200 --warmup 20; } > $D/bench_driver_cmd.log 2>&1
{ echo '$ python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpus 2 --no-cpu'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpus 2 --no-cpu; } > $D/cpus2.log 2>&1
