#!/bin/bash
# Block-row order of the column-stream kernels (SPMM_BSR_ORDER: 0 auto,
# 1 longest first, 2 XCD-chunked) x variants, after the BSR parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_scale.py -x -q --timeout 120 --timeout-method thread -k "not hybrid" > gpurun_out/order_tests.log 2>&1; rc=$?
tail -2 gpurun_out/order_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/order_tests.log | head -20; exit 1; }
: > gpurun_out/order_sweep.jsonl
for w in ${BW:-reddit_bsr32 reddit_rcm_bsr32 products_bsr32 products_bsr16_f16}; do
  for o in ${ORDERS:-2 1}; do
    for v in ${VARS:-4596 4556}; do
      case $w in *bsr16*) v=5021;; esac
      SPMM_BSR_ORDER=$o SPMM_BSR_VARIANT=$v timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
      grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); r['variant']=$v; r['order']=$o; print(json.dumps(r))" >> gpurun_out/order_sweep.jsonl
      grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', 'order', $o, 'var', $v, r['ms_per_step'], r['roofline'].get('kernel_ms'))"
      case $w in *bsr16*) break;; esac
    done
  done
done
