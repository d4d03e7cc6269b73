# round 6: phase and per-chunk stamps of the layer, pair operands (variant 13) and register-staged (0), WD_STAMPS build
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r6s
for v in 13 0; do
  WD_VARIANT=$v WDMPNN_LIB=$PWD/exp/libwdmpnn_pst2.so timeout -k 10 300 python3 -u tools/stamps_layer.py > gpurun_out/r6s/stamps2_v$v.log 2>&1
done
