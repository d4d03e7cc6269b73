# round 6: the restructured pair-operand loop in the product library -- the pair-path GPU tests, then the
# driver's bench command on the default path and on gemm_variant 13 (pair operands), one box, and the
# rocprofv3 kernel stats of the headline workload with one batch in flight for both
set -e
export TMPDIR=/tmp
D=gpurun_out/r6q
mkdir -p $D
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "pair or one_launch or golden" > $D/pytest_pairs.log 2>&1
for v in 0 13; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --variant $v --stream-train-graphs 0 > $D/bench_v$v.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_v$v -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 --variant $v > $D/prof_v$v.log 2>&1
  python3 tools/kstats.py $D/prof_v$v/run_kernel_stats.csv 8 > $D/kstats_v$v.txt
done
