#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_bsr.py -x -q > gpurun_out/pytest_bsr.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_bsr.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|mismatch" gpurun_out/pytest_bsr.log | head -30; exit $rc; }
WL=products_bsr16_f16 VARS="4099 4100 4102 12" bash tools/bsr_variants.sh || exit 1
WL=products_bsr16_f16 EXTRA="--dtype fp32" VARS="4099 4100 4102 8" bash tools/bsr_variants.sh || exit 1
WL=products_bsr32 VARS="4099 4107" bash tools/bsr_variants.sh || exit 1
