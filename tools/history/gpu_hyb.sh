#!/bin/bash
# Hybrid BSR-part kernel and threshold sweep: HV = variants, HD = densities.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${HW:-reddit_hybrid32 products_hybrid32}; do
  for v in ${HV:-4124 4225}; do
    for d in ${HD:-auto}; do
      SPMM_BSR_VARIANT=$v timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --density $d > gpurun_out/hy.log 2>&1 || { tail -5 gpurun_out/hy.log; exit 1; }
      grep '^{' gpurun_out/hy.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['config']; print('$w', 'var=$v', 'd=$d', c['nnzb'], c['csr_remainder_nnz'], r['ms_per_step'], r.get('part_kernel_ms'))"
    done
  done
done
