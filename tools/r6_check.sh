# round 6: GPU suite, smoke, the driver's bench command, and the same command on 2 CPUs (--cpus 2: one
# rank's share when 8 ranks share a 16-CPU quota); in-tree library
set -e
export TMPDIR=/tmp
D=gpurun_out/r6
mkdir -p $D
rc=0; timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $D/pytest_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1
{ echo '$ python3 bench.py --gpus 1 --steps 20 --warmup 5'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5; } > $D/bench_driver_cmd.log 2>&1
{ echo '$ python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpus 2 --no-cpu'; timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpus 2 --no-cpu; } > $D/bench_cpus2.log 2>&1
exit $rc
