#!/bin/bash
# same-box training-step A/B of experiment libraries: ms per step (tools/train_bench.py, twice each) and one
# step's kernel trace per library under rocprofv3.  LIBS="a b" bash tools/train_ab_libs.sh
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for v in $LIBS; do
    WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/tab_$v.log 2>&1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4))" gpurun_out/tab_$v.log $v
  done
done
for v in $LIBS; do
  WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tabprof_$v -o run -- python3 tools/train_bench.py > /dev/null 2>&1
  python tools/train_trace_db.py gpurun_out/tabprof_$v/run_results.db > gpurun_out/tabtrace_$v.txt
done
