#!/bin/bash
# Fused hybrid with the longest-first block-row order: parity, then the
# hybrid workloads with SPMM_BSR_ORDER 2 (XCD chunks) / 1 (longest first),
# and the RCM-reordered reddit forced fused (--hybrid-options 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bsr.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread > gpurun_out/hyb_tests.log 2>&1; rc=$?
tail -2 gpurun_out/hyb_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/hyb_tests.log | head -20; exit 1; }
: > gpurun_out/hyb_order_sweep.jsonl
run() {  # workload order extra...
  w=$1; o=$2; shift 2
  SPMM_BSR_ORDER=$o timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
  grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); r['order']=$o; r['extra']='$*'; print(json.dumps(r))" >> gpurun_out/hyb_order_sweep.jsonl
  grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', 'order', $o, '$*', r['ms_per_step'], r.get('part_kernel_ms'), r['config'].get('fused'))"
}
for o in 2 1; do run reddit_hybrid32 $o; done
for o in 2 1; do run products_hybrid32 $o; done
for o in 2 1; do run reddit_rcm_hybrid32 $o --hybrid-options 1; done
run reddit_rcm_hybrid32 0
