#!/bin/bash
# GPU-box driver for one gpurun call: each GPU step has its own time limit; any exit code other than
# 0 (ok) or 1 (test failures) stops the call (fault / abort / timeout => start nothing more on the GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchq) step bench_quick 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 5 ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --stream-graphs 0 --stream-train-graphs 0 ;;
    lab) step gemm_lab 300 ./tools/gemm_lab 200 ;;
    stream) step stream 120 ./tools/gemm_lab 50 stream ;;
    mainloop) step mainloop 120 ./tools/gemm_lab 200 mainloop ;;
    train) step train 300 python tools/train_bench.py ;;
    proftrain) step rocprof_train 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_train -o run --output-format csv -- python tools/train_bench.py ;;
    host) step host 300 python tools/host_overhead.py ;;
    hiptrace) step hiptrace 300 rocprofv3 --hip-trace --stats --output-format csv -d gpurun_out/hiptrace -o run -- python tools/host_overhead.py ;;
    packprof) step pack_profile 200 python tools/pack_profile.py ;;
    ab) step ab_x6 300 python bench.py --steps 200 --warmup 20 --no-cpu --variant 10 && step ab_f32 300 python bench.py --steps 200 --warmup 20 --no-cpu --variant 9 ;;
    x6prec) step x6prec 300 python tools/x6_precision.py ;;
    profx6) step rocprof_x6 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_x6 -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --variant ${VARIANT:-10} ;;
    counters) step counters 120 rocprofv3 -L ;;
    pmc) step pmc 1500 bash tools/pmc.sh ;;
    profqm9) step rocprof_qm9 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_qm9 -o run --output-format csv -- python bench.py --kind qm9 --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --stream-graphs 0 --stream-train-graphs 0 ;;
    sweep) step sweep 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sweep -o run -- python tools/size_sweep.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
