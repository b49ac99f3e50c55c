#!/bin/bash
# Column-masked BSR kernels: parity for each variant in CMP (forced through
# SPMM_BSR_VARIANT), then timings of each variant in CMV on each workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for V in ${CMP:-4200}; do
  SPMM_BSR_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 120 --timeout-method thread \
    -k "${CMK:-column_sparse or lds_staged or mfma_shapes}" > gpurun_out/cm_pt.log 2>&1; rc=$?
  echo "parity var=$V: $(tail -1 gpurun_out/cm_pt.log)"
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/cm_pt.log | head -20; exit 1; }
done
for w in ${CMW:-reddit_bsr32 products_bsr32}; do
  for v in ${CMV:-4200}; do
    SPMM_BSR_VARIANT=$v timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 ${CMB:-} > gpurun_out/cm_b.log 2>&1 || { tail -5 gpurun_out/cm_b.log; exit 1; }
    grep '^{' gpurun_out/cm_b.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', 'var=$v', r['ms_per_step'], r['roofline'].get('kernel_ms'), 'csr', r.get('csr_same_matrix_ms'))"
  done
done
