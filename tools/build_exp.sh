#!/bin/bash
# Experiment library: bash tools/build_exp.sh NAME [-DMACRO=V ...] -> exp/libwdmpnn_NAME.so (A/B with WDMPNN_LIB)
# Compiles a snapshot of the sources: hipcc's device and host passes read the files separately, and a
# source edited between them once gave a library whose host code launched a kernel its code object lacked
# (round 5: slab_reduce_multi_kernel, DESIGN.md §4 "Load-time kernel check").
set -e
cd "$(dirname "$0")/.."
name=$1; shift
snap=$(mktemp -d /tmp/wdmpnn_exp_XXXXXX)
trap 'rm -rf "$snap"' EXIT
cp -r include polymer-chemprop_amd/csrc "$snap"/
mkdir -p exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function "$@" \
    -I "$snap/include" -I "$snap/csrc" "$snap/csrc/wdmpnn.hip" -o exp/libwdmpnn_$name.so
echo "built exp/libwdmpnn_$name.so"
