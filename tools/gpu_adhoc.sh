#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_csr.py -x -q -k "shards or permutation" > gpurun_out/pt.log 2>&1; rc=$?
tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || grep -E "Error|assert" gpurun_out/pt.log | head
