#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_convert.py -x -q -s > gpurun_out/conv.log 2>&1; rc=$?
grep -E "passed|failed|device csr2bsr|Error|assert" gpurun_out/conv.log | head -20
exit $rc
