#!/bin/bash
# same-box A/B of the training step (tools/train_bench.py) across experiment libraries (WDMPNN_LIB):
#   bash tools/train_ab.sh base cur
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2 3; do
  for v in "$@"; do
    export WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so
    timeout -k 10 200 python tools/train_bench.py > gpurun_out/tab_$v.log 2>&1 || exit $?
    python - "$v" <<'PY'
import json,sys
l=[x for x in open(f'gpurun_out/tab_{sys.argv[1]}.log') if x.startswith('{')][-1]; d=json.loads(l)
print(sys.argv[1], 'ms/step', round(d['ms_per_step'], 4))
PY
  done
done
