#!/bin/bash
# bs = 32 column stream: O32 variants (455P) against the shipped 4596, parity
# under the candidate, then the bs 32 workloads per variant (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V0=${V0:-4556}
SPMM_BSR_VARIANT=$V0 timeout -k 10 600 python -u -m pytest tests/test_gpu_bsr.py -x -q --timeout 120 --timeout-method thread -k "not hybrid" > gpurun_out/cs2o_tests.log 2>&1; rc=$?
tail -2 gpurun_out/cs2o_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/cs2o_tests.log | head -20; exit 1; }
: > gpurun_out/cs2o_sweep.jsonl
for w in ${BW:-reddit_bsr32 products_bsr32}; do
  for v in ${VARS:-4596 4556 4558 4554 4596}; do
    SPMM_BSR_VARIANT=$v timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bw.log 2>&1 || { tail -5 gpurun_out/bw.log; exit 1; }
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); r['variant']=$v; print(json.dumps(r))" >> gpurun_out/cs2o_sweep.jsonl
    grep '^{' gpurun_out/bw.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w', $v, r['ms_per_step'], r['roofline'].get('kernel_ms'))"
  done
done
