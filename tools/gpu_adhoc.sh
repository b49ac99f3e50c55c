#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
hb() {  # workload, label, args
  local w=$1 lab=$2; shift 2
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/h.log 2>&1 || { tail -5 gpurun_out/h.log; exit 1; }
  grep '^{' gpurun_out/h.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w $lab', r['ms_per_step'], r.get('part_kernel_ms'), r['roofline'].get('kernel_ms'), r.get('csr_same_matrix_ms'))"
}
for o in 1 5 1 5; do
  hb products_csr o$o --csr-options $o
  hb arxiv_csr o$o --csr-options $o
  hb reddit_hybrid32 o$o --csr-options $o
  hb reddit_rcm_hybrid32 o$o --csr-options $o
done
