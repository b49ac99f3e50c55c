#!/bin/bash
# The pair column stream (bs 16 fp16, SPMM_BSR_VARIANT=6504): BSR parity subset and
# the full-scale bs 16 tests under it, then interleaved timings against the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${V:-6504}
SPMM_BSR_VARIANT=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread -k "${PYTEST_EXPR:-not hybrid and not reddit_scale and not 32}" > gpurun_out/pcs_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pcs_tests.log
[ $rc -ge 124 ] && exit $rc
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pcs_tests.log | head -20; exit 1; }
RUNS="${RUNS:-products_bsr16_f16:d products_bsr16_f16:$V products_rcm_bsr16_f16:d products_rcm_bsr16_f16:$V}" REPS=${REPS:-2} bash tools/gpu_var.sh
