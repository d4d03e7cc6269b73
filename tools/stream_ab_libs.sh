#!/bin/bash
# same-box A/B of the streamed leg (configs[4]) for experiment libraries: bash tools/stream_ab_libs.sh cur fg
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in ${ROUNDS:-1 2}; do
  for v in "$@"; do
    export WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-secondary --many 0 --stream-graphs 300000 \
      --stream-train-graphs 16384 $SAB_ARGS > gpurun_out/sab_$v${SAB_TAG}.log 2>&1 || exit $?
    python - "$v" "$SAB_TAG" <<'PY'
import json,sys
l=[x for x in open(f"gpurun_out/sab_{sys.argv[1]}{sys.argv[2]}.log") if x.startswith('{')][-1]; d=json.loads(l)
print(f"{sys.argv[1]:8s} streamed {d['streamed']['value']/1e6:7.2f} M edges/s  streamed training {d['streamed_training']['ms_per_step']:.3f} ms/step")
PY
  done
done
