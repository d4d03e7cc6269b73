# round 6: stage-by-stage decode of the pair-operand forward (tools/debug_pairs.py) with exp/libwdmpnn_pairs3.so
set -e
export TMPDIR=/tmp
export WDMPNN_LIB=$PWD/exp/libwdmpnn_pairs3.so
mkdir -p gpurun_out/r6d
timeout -k 10 300 python3 -u tools/debug_pairs.py polymer 64 300 > gpurun_out/r6d/debug.log 2>&1
