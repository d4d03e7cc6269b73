#!/bin/bash
# Experiment library: bash tools/build_exp.sh NAME [-DMACRO=V ...] -> exp/libwdmpnn_NAME.so (A/B with WDMPNN_LIB)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function "$@" \
    -I include -I polymer-chemprop_amd/csrc polymer-chemprop_amd/csrc/wdmpnn.hip -o exp/libwdmpnn_$name.so
echo "built exp/libwdmpnn_$name.so"
