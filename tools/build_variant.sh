#!/bin/bash
# A/B builds of the library with compile-time switches: tools/build_variant.sh NAME "-DFLAG=V ..."
# builds out of tree in /tmp/var_NAME and installs spmm-denseblock_amd/lib_var/NAME.so (swapped
# over lib/libspmm_hip.so on the GPU box by the timing script; never the release library).
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; F=${2:-}
T=/tmp/var_$N
mkdir -p "$T/csrc" "$T/include"
cp "$R"/spmm-denseblock_amd/csrc/* "$T/csrc/"
cp "$R"/include/* "$T/include/"
cp "$R/spmm-denseblock_amd/Makefile" "$T/"
make -C "$T" -j8 ROOT="$T" HIPCC="/opt/rocm/bin/hipcc $F" lib > "$T/build.log" 2>&1 || { tail -20 "$T/build.log"; exit 1; }
mkdir -p "$R/spmm-denseblock_amd/lib_var"
cp "$T/lib/libspmm_hip.so" "$R/spmm-denseblock_amd/lib_var/$N.so"
echo "$N: $F"
