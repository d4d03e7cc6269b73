set -e
export TMPDIR=/tmp
for v in ${LIBS:-base ae1 ae4 ae7}; do
  WDMPNN_LIB=$PWD/exp/libwdmpnn_$v.so STEPS=20 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/adprof_$v -o run -- python3 tools/train_bench.py > /dev/null 2>&1
done
