#!/bin/bash
# BSR path after a kernel change: all BSR/scale/convert GPU tests, then every
# BSR / hybrid bench workload once (kernel ms and step ms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_scale.py tests/test_gpu_convert.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bsr_tests.log 2>&1; rc=$?
tail -2 gpurun_out/bsr_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/bsr_tests.log | head -20; exit 1; }
: > gpurun_out/bsr_sweep.jsonl
for w in ${BW:-reddit_bsr32 products_bsr32 products_bsr16_f16 reddit_hybrid32 products_hybrid32 reddit_rcm_hybrid32}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
  grep '^{' gpurun_out/bw.log >> gpurun_out/bsr_sweep.jsonl
  grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', r['ms_per_step'], r['roofline'].get('kernel_ms'), r.get('part_kernel_ms'), 'csr', r.get('csr_same_matrix_ms'))"
done
