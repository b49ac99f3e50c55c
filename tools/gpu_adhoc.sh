#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_csr.py tests/test_gpu_bsr.py -x -q > gpurun_out/pt.log 2>&1; rc=$?
tail -1 gpurun_out/pt.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|mismatch" gpurun_out/pt.log | head -30; exit 1; }
for K in 48 64; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --K $K > gpurun_out/h.log 2>&1 || { tail -5 gpurun_out/h.log; exit 1; }
  grep '^{' gpurun_out/h.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('K=$K', r['ms_per_step'], r['roofline'].get('kernel_ms'), r['roofline'].get('frac'))"
done
