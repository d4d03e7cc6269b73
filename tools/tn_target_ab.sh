# training step vs the TN GEMMs' split target (WDMPNN_TN_TARGET workgroups), same box, two passes
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in 512 384 768 1024; do
    WDMPNN_TN_TARGET=$v timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/tnt_$v.log 2>&1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('target', sys.argv[2], round(d['ms_per_step'],4))" gpurun_out/tnt_$v.log $v
  done
done
