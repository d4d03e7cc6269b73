# round 6 closing evidence on one box with the final tree: the GPU suite, smoke, host breakdown, profiles
# (rocprof one / three streams, PMC, training trace), then the driver's bench command and the two-CPU run
set -e
export TMPDIR=/tmp
D=gpurun_out/r6l
mkdir -p $D
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $D/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1
timeout -k 10 200 python3 -u tools/host_breakdown.py polymer > $D/host_breakdown.log 2>&1
timeout -k 10 200 python3 -u tools/host_breakdown.py qm9 >> $D/host_breakdown.log 2>&1
rm -rf gpurun_out/pmc gpurun_out/r6e
bash tools/r6_prof.sh
bash tools/r6_bench2.sh
