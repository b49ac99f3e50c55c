#!/bin/bash
# bs 16 fp16 column-stream / item-stream variants on one GPU box: digests of C
# against the column stream (bit-identical by construction), the BSR parity
# tests under one variant, then the config-5 workload per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/is16_digests.log
for v in ${DV:-6104 5021}; do
  SPMM_BSR_VARIANT=$v timeout -k 10 300 python tools/is16_check.py >> gpurun_out/is16_digests.log 2>&1 || { tail -5 gpurun_out/is16_digests.log; exit 1; }
done
cat gpurun_out/is16_digests.log
V0=${V0:-6104} VARS="${VARS:-6104 6121 5021 5533 5910}" bash tools/gpu_cs16.sh
