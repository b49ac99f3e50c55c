#!/bin/bash
# BSR MFMA kernel variant sweep (SPMM_BSR_VARIANT, csrc/bsr_kernels.hip):
# VAR & 3 = pipeline, VAR & 4 = XCD remap (bs 32), VAR >> 3 = min waves/SIMD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS:-40 44 42}; do
  SPMM_BSR_VARIANT=$v timeout -k 10 300 python bench.py --workload ${WL:-reddit_bsr32} ${EXTRA:-} --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/v.log 2>&1 || { tail -20 gpurun_out/v.log; exit 1; }
  grep '^{' gpurun_out/v.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$WL $v', r['roofline']['kernel_ms'], r['roofline']['achieved'], r['roofline']['frac'])"
done
