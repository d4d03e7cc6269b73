#!/bin/bash
# streamed workloads (configs[4]) vs the number of native producer threads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for p in 4 8 12; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-secondary --stream-graphs 200000 \
      --stream-train-graphs 32768 --producers $p > gpurun_out/stream_p$p.log 2>&1 || exit $?
  python - "$p" <<'PY'
import json,sys
l=[x for x in open(f'gpurun_out/stream_p{sys.argv[1]}.log') if x.startswith('{')][-1]; d=json.loads(l)
print('producers', sys.argv[1], 'streamed M edges/s', round(d['streamed']['value']/1e6,2),
      'streamed training ms/step', round(d['streamed_training']['ms_per_step'],3))
PY
done
