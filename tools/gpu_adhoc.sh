#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pt_all.log 2>&1; rc=$?
tail -3 gpurun_out/pt_all.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|mismatch" gpurun_out/pt_all.log | head -30; exit 1; }
