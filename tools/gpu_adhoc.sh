#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SPMM_BSR_VARIANT=4303 timeout -k 10 300 python -m pytest tests/test_gpu_bsr.py -x -q -k "16-f16 or test_bsrmm_f16" > gpurun_out/pt.log 2>&1; rc=$?
echo "$(tail -1 gpurun_out/pt.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pt.log | head; exit 1; }
WL=products_bsr16_f16 VARS="4107 4303 4304 4107 4303" bash tools/bsr_variants.sh || exit 1
