# in-tree library: GPU suite, the training step twice (tools/train_bench.py) and one step's kernel trace
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tc_pytest.log 2>&1
tail -1 gpurun_out/tc_pytest.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/tc_$r.log 2>&1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('step ms', round(d['ms_per_step'],4))" gpurun_out/tc_$r.log
done
STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tcprof -o run -- python3 tools/train_bench.py > /dev/null 2>&1
python tools/train_trace_db.py gpurun_out/tcprof/run_results.db > gpurun_out/tctrace.txt
