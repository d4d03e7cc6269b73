#!/bin/bash
# Kernel-time A/B of experiment builds (gpurun_exp_<n>.so, built with -DWD_EXP=<n>) vs the product library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/exp
for v in prod ${EXPS-1 2 3}; do
  lib=polymer-chemprop_amd/chemprop_amd/libwdmpnn.so
  [ "$v" != prod ] && lib=$PWD/gpurun_exp_$v.so
  WDMPNN_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp/$v${EXP_TAG:-} -o run -- \
      python bench.py --steps 100 --warmup 10 --no-cpu --no-secondary --streams 1 --stream-graphs 0 --stream-train-graphs 0 ${EXP_BENCH_ARGS:-} > gpurun_out/exp/$v${EXP_TAG:-}.log 2>&1 || { echo "exp $v failed"; tail -5 gpurun_out/exp/$v${EXP_TAG:-}.log; exit 1; }
  echo "== $v  $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/exp/$v${EXP_TAG:-}.log)"
  python3 -c "
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:5]:
    print(f\"  {r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:8.2f} us\")" gpurun_out/exp/$v${EXP_TAG:-}/run_kernel_stats.csv
done
