#!/bin/bash
# same-box A/B of experiment libraries (exp/libwdmpnn_<name>.so, WDMPNN_LIB) against each other:
#   bash tools/ab_libs.sh base w81 w15
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 300 --warmup 20 --no-cpu --stream-graphs 0 --stream-train-graphs 0 --no-secondary --many 0"
for round in 1 2; do
  for v in "$@"; do
    export WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so
    timeout -k 10 200 $B > gpurun_out/abl_$v.log 2>&1 || exit $?
    python - "$v" <<'PY'
import json,sys
l=[x for x in open(f'gpurun_out/abl_{sys.argv[1]}.log') if x.startswith('{')][-1]; d=json.loads(l)
print(sys.argv[1], round(d['value']/1e6,2), 'single', round(d['single_stream']['value']/1e6,2), 'layer us', round(d['roofline']['avg_launch_us'],2))
PY
  done
done
