# training-step A/B of experiment libraries (ms per step) + TN kernel times under rocprofv3
set -e
export TMPDIR=/tmp
for v in ${LIBS:-base tn3 tn4}; do
  for tgt in ${TARGETS:-512}; do
    WDMPNN_TN_TARGET=$tgt WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so timeout -k 10 200 python -u tools/train_bench.py > gpurun_out/tnab_${v}_$tgt.log 2>&1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],4))" gpurun_out/tnab_${v}_$tgt.log $v $tgt
    WDMPNN_TN_TARGET=$tgt WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tnprof_${v}_$tgt -o run -- python3 tools/train_bench.py > /dev/null 2>&1
  done
done
