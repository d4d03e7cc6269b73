# round 6: the pair-operand library (exp/libwdmpnn_pairs4.so): the GPU suite (every failure listed), then the
# driver's bench command with it (pairs) and with gemm_variant 12 (register-staged layers), one box, and the
# rocprofv3 kernel stats of the headline workload with one batch in flight
set -e
export TMPDIR=/tmp
export WDMPNN_LIB=$PWD/exp/libwdmpnn_pairs4.so
D=gpurun_out/r6p
mkdir -p $D
# (test failures, exit 1, do not stop the script; a crash or time-out does)
rc=0; timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $D/pytest_gpu.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 0 12; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --variant $v --stream-train-graphs 0 > $D/bench_v$v.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 > $D/prof.log 2>&1
python3 tools/kstats.py $D/prof/run_kernel_stats.csv 8 > $D/kstats.txt
