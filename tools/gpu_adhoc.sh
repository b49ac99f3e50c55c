#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
hb() {  # workload, label, args
  local w=$1 lab=$2; shift 2
  timeout -k 10 300 python bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/h.log 2>&1 || { tail -5 gpurun_out/h.log; exit 1; }
  grep '^{' gpurun_out/h.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$w $lab', r['ms_per_step'], r['roofline'].get('kernel_ms'), r['roofline'].get('frac'))"
}
for wpc in 16 24 32; do
  hb arxiv_csr w$wpc --waves-per-cu $wpc
  hb arxiv_csr w$wpc-graph --waves-per-cu $wpc --graph
done
hb products_csr graph --graph
