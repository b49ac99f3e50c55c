#!/bin/bash
# Column-stream bs = 32 kernel (variants 45PA) on one GPU box: the BSR parity
# tests under the variant, then the bs = 32 bench workloads per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V0=${V0:-4583}
SPMM_BSR_VARIANT=$V0 timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_EXPR:-not hybrid_fused_vs_two}" > gpurun_out/cs_tests.log 2>&1; rc=$?
tail -3 gpurun_out/cs_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/cs_tests.log | head -20; exit 1; }
: > gpurun_out/cs_sweep.jsonl
for w in ${BW:-reddit_bsr32 products_bsr32}; do
  for v in ${VARS:-4402 4583 4584 4543 4563 4582}; do
    SPMM_BSR_VARIANT=$v timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); r['variant']=$v; print(json.dumps(r))" >> gpurun_out/cs_sweep.jsonl
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', $v, r['ms_per_step'], r['roofline'].get('kernel_ms'), 'csr', r.get('csr_same_matrix_ms'))"
  done
done
