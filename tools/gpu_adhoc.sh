#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in reddit_hybrid32 products_hybrid32; do
  for bs in 16 32; do
    for d in auto 0.0625 0.125; do
      timeout -k 10 300 python bench.py --workload $wl --bs $bs --density $d --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/h.log 2>&1 || { tail -20 gpurun_out/h.log; exit 1; }
      grep '^{' gpurun_out/h.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['config']; print('$wl bs=$bs d=$d', r['ms_per_step'], r['part_kernel_ms'], c['nnzb'], c['csr_remainder_nnz'], (r.get('plan') or {}).get('density'))"
    done
  done
done
