#!/bin/bash
# same-box A/B of experiment libraries on the three forward modes: two streams, one stream, forward_many(4)
#   bash tools/ab3.sh cur wo1 e80
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python bench.py --steps 400 --warmup 20 --no-cpu --stream-graphs 0 --stream-train-graphs 0 --no-secondary --many 4"
for round in 1 2; do
  for v in "$@"; do
    export WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so
    timeout -k 10 200 $B > gpurun_out/ab3_$v.log 2>&1 || exit $?
    python - "$v" <<'PY'
import json,sys
l=[x for x in open(f'gpurun_out/ab3_{sys.argv[1]}.log') if x.startswith('{')][-1]; d=json.loads(l)
print(f"{sys.argv[1]:8s} two-stream {d['value']/1e6:7.2f}  single {d['single_stream']['value']/1e6:7.2f}  many4 {d['forward_many']['value']/1e6:7.2f}  layer {d['roofline']['avg_launch_us']:6.2f} us")
PY
  done
done
