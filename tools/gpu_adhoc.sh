#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_csr.py -x -q > gpurun_out/pt_csr.log 2>&1; rc=$?
tail -2 gpurun_out/pt_csr.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|mismatch" gpurun_out/pt_csr.log | head -20; exit 1; }
for K in 32 16 8 4; do
    timeout -k 10 300 python bench.py --K $K --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/k.log 2>&1 || { tail -5 gpurun_out/k.log; exit 1; }
    grep '^{' gpurun_out/k.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('K=$K', r['roofline']['kernel_ms'], r['roofline']['frac'], r['ms_per_step'])"
done
