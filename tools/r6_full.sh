# round 6: the GPU suite (failures listed, not stopping), smoke, the driver's bench command and the rocprofv3
# kernel stats of the headline workload (one batch in flight) with the in-tree library
set -e
export TMPDIR=/tmp
D=gpurun_out/r6f
mkdir -p $D
rc=0; timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $D/pytest_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 > $D/prof.log 2>&1
python3 tools/kstats.py $D/prof/run_kernel_stats.csv 8 > $D/kstats.txt
exit $rc
