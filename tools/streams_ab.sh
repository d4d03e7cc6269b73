#!/bin/bash
# batches in flight sensitivity (same box, ABAB): the default bench leg with --streams 1..4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for round in 1 2; do
  for n in 2 3 4; do
    timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-cpu --no-secondary --stream-graphs 0 --stream-train-graphs 0 --many 0 --streams $n > gpurun_out/streams_$n.log 2>&1 || exit $?
    python - "$n" <<'PY'
import json,sys
l=[x for x in open(f'gpurun_out/streams_{sys.argv[1]}.log') if x.startswith('{')][-1]; d=json.loads(l)
print(f"streams {sys.argv[1]}: {d['value']/1e6:7.2f} M edges/s ({d['ms_per_step']*1e3:5.1f} us/step)")
PY
  done
done
