#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_bsr.py -x -q > gpurun_out/pytest_bsr.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_bsr.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_bsr.log | head -20; exit $rc; }
for v in 4099 4098 4100 4107 40; do
  SPMM_BSR_VARIANT=$v timeout -k 10 300 python tools/bsr_micro.py || exit 1
done
WL=reddit_bsr32 VARS="4099 4098 4100 4107" bash tools/bsr_variants.sh || exit 1
WL=products_bsr32 VARS="4099 4098" bash tools/bsr_variants.sh || exit 1
for wl in reddit_hybrid32 products_hybrid32; do
    timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/hyb.log 2>&1 || { tail -20 gpurun_out/hyb.log; exit 1; }
    grep '^{' gpurun_out/hyb.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['config']; print('$wl', r['ms_per_step'], r['part_kernel_ms'])"
done
