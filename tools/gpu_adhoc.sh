#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 4107 4172 4188 4164; do
  SPMM_BSR_VARIANT=$v timeout -k 10 300 python tools/bsr_micro.py || exit 1
done
WL=reddit_bsr32 VARS="4107 4172" bash tools/bsr_variants.sh || exit 1
SPMM_BSR_VARIANT=4172 timeout -k 10 400 python -m pytest tests/test_gpu_bsr.py -x -q -k "lds or mfma_shapes or hybrid" > gpurun_out/pt.log 2>&1; tail -2 gpurun_out/pt.log
