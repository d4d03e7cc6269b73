set -e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "repack or direct or adam or training" > gpurun_out/pytest_repack.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/tb_repack.log 2>&1
  NO_REPACK=1 timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/tb_norepack.log 2>&1
  for f in repack norepack; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4))" gpurun_out/tb_$f.log $f; done
done
STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/rocprof_train6 -o run -- python3 tools/train_bench.py > gpurun_out/train_prof_v6.log 2>&1
LIBS="tnnomax" bash tools/r5_tn.sh
