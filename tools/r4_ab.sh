#!/bin/bash
# Round-4 GPU session: parity tests of the in-tree library, then a same-box A/B of experiment libraries
# (exp/libwdmpnn_<name>.so) and a rocprof kernel summary of the in-tree one.
#   bash tools/r4_ab.sh base s2 s3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_libs.sh "$@" || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_ab -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 > gpurun_out/rocprof_ab.log 2>&1 && python tools/kstats.py gpurun_out/rocprof_ab/run_kernel_stats.csv 6
