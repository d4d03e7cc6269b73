#!/bin/bash
# bench value vs batches in flight (HIP streams), same box, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for s in 2 3 2 3 4; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu --no-secondary --stream-graphs 0 \
      --stream-train-graphs 0 --streams $s > gpurun_out/streams_$s.log 2>&1 || exit $?
  python - "$s" <<'PY'
import json,sys
l=[x for x in open(f'gpurun_out/streams_{sys.argv[1]}.log') if x.startswith('{')][-1]; d=json.loads(l)
print('streams', sys.argv[1], round(d['value']/1e6,2), 'single', round(d['single_stream']['value']/1e6,2))
PY
done
