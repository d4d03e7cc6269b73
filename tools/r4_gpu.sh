#!/bin/bash
# Round-4 GPU session driver: each step under its own limit, stop at the first fault/timeout.
#   bash tools/r3_gpu.sh tests lab ab prof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T): $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)"
  tail -n ${TAILN:-15} "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    testsv) step pytest_gpu 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    lab) step lab_mainloop 150 ./tools/gemm_lab 200 mainloop ;;
    ab) step ab 600 bash tools/ab_libs.sh ${AB:-base cur} ;;
    ab3) step ab3 900 bash tools/ab3.sh ${AB3:-cur base} ;;
    bench) step bench 600 python bench.py ;;
    benchq) step benchq 300 python bench.py --steps 200 --warmup 20 --no-cpu --no-secondary --stream-graphs 0 --stream-train-graphs 0 ;;
    prof) step rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 && python tools/kstats.py gpurun_out/rocprof/run_kernel_stats.csv 8 ;;
    pmc) step pmc 900 bash tools/pmc.sh && python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_traffic.json > gpurun_out/pmc_summary.txt ;;
    train) step train 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_train -o run --output-format csv -- python tools/train_bench.py && python tools/train_trace.py gpurun_out/rocprof_train/run_kernel_trace.csv > gpurun_out/train_trace.txt && tail -3 gpurun_out/train_trace.txt ;;
    stream) step stream 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_stream -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-secondary --stream-graphs 200000 --stream-train-graphs 0 && python tools/kstats.py gpurun_out/rocprof_stream/run_kernel_stats.csv 8 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
