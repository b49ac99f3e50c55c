#!/bin/bash
# Builds the TUNING A/B library (make TUNING=1: SPMM_BSR_VARIANT / SPMM_GRP_VARIANT / ... read
# from the environment) out of tree in ${TUN:-/tmp/tun}, audits its column-stream kernels for
# compiler touches of in-flight asm-load registers (tools/isa_vmcnt.py --inflight: a spilled row
# index is an illegal address on the GPU), and only then installs it as
# spmm-denseblock_amd/lib_tuning/libspmm_hip.so (copied over lib/ on the box by the sweep scripts).
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
T=${TUN:-/tmp/tun}
mkdir -p "$T/csrc" "$T/include"
cp "$R"/spmm-denseblock_amd/csrc/* "$T/csrc/"
cp "$R"/include/* "$T/include/"
cp "$R/spmm-denseblock_amd/Makefile" "$T/"
make -C "$T" -j8 TUNING=1 ROOT="$T" lib > "$T/build.log" 2>&1 || { tail -20 "$T/build.log"; exit 1; }
python3 "$R/tools/isa_vmcnt.py" --inflight "$T/build/bsr_kernels-hip-amdgcn-amd-amdhsa-gfx950.s" > "$T/inflight.txt" || {
  grep -v '^ok' "$T/inflight.txt"; echo "TUNING build NOT installed"; exit 1; }
mkdir -p "$R/spmm-denseblock_amd/lib_tuning"
cp "$T/lib/libspmm_hip.so" "$R/spmm-denseblock_amd/lib_tuning/libspmm_hip.so"
tail -1 "$T/inflight.txt"
