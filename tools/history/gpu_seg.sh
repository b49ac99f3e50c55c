#!/bin/bash
# Block-row segments of the bs 32 column stream: parity (small tests split rows
# past 64 blocks; scale tests), then reddit / RCM reddit / products with
# SPMM_BSR_ORDER 0 (auto: segments on shallow grids), 3 (longest first, no
# split), 2 (XCD order).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/seg_tests.log 2>&1; rc=$?
tail -2 gpurun_out/seg_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/seg_tests.log | head -20; exit 1; }
: > gpurun_out/seg_sweep.jsonl
for w in ${BW:-reddit_bsr32 reddit_rcm_bsr32 products_bsr32}; do
  for o in ${ORDERS:-0 3 2 0}; do
    SPMM_BSR_ORDER=$o timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); r['order']=$o; print(json.dumps(r))" >> gpurun_out/seg_sweep.jsonl
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', 'order', $o, r['ms_per_step'], r['roofline'].get('kernel_ms'))"
  done
done
