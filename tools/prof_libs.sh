#!/bin/bash
# rocprof kernel summary (one batch in flight) of experiment libraries exp/libwdmpnn_<name>.so, one after
# another on the same box:   bash tools/prof_libs.sh cur nogemm
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  export WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --many 0 --stream-graphs 0 --stream-train-graphs 0 ${PROF_ARGS:-} > gpurun_out/prof_$v.log 2>&1 || exit $?
  echo "== $v"; python tools/kstats.py gpurun_out/prof_$v/run_kernel_stats.csv 4
done
