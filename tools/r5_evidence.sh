# round-end evidence on one box: full GPU suite, smoke, the driver's bench command next to a 200-step run,
# rocprofv3 kernel statistics of the headline workload (single stream)
set -e
export TMPDIR=/tmp
D=gpurun_out/ev
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ > $D/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1
{ echo '$ python3 bench.py --gpus 1 --steps 20 --warmup 5'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5;
  echo '$ python3 bench.py --gpus 1 --steps 200 --warmup 20'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 200 --warmup 20; } > $D/bench_driver_cmd.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 > $D/prof.log 2>&1
STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d $D/train -o run -- python3 tools/train_bench.py > $D/train_prof.log 2>&1
python tools/train_trace_db.py $D/train/run_results.db > $D/train_trace.txt
