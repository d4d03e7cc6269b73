# round 6: per-workgroup phase stamps and per-chunk loop stamps of the pair-operand layer (WD_STAMPS build)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r6s
WDMPNN_LIB=$PWD/exp/libwdmpnn_pstamps.so timeout -k 10 300 python3 -u tools/stamps_layer.py > gpurun_out/r6s/stamps_pairs.log 2>&1
