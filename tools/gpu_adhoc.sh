#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_bsr.py -x -q > gpurun_out/pt_bsr.log 2>&1; rc=$?
tail -1 gpurun_out/pt_bsr.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|mismatch" gpurun_out/pt_bsr.log | head -30; exit 1; }
hb() {  # workload, label, env/args
  local w=$1 lab=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline $HOPT > gpurun_out/h.log 2>&1 || { tail -5 gpurun_out/h.log; exit 1; }
  grep '^{' gpurun_out/h.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w $lab', r['ms_per_step'], r.get('part_kernel_ms'), r['roofline'].get('kernel_ms'))"
}
for w in reddit_hybrid32 products_hybrid32 reddit_rcm_hybrid32 reddit_bsr32 products_bsr32; do
  for v in 4107 4123 4124 4125; do
    HOPT=""; hb $w v$v SPMM_BSR_VARIANT=$v
  done
done
